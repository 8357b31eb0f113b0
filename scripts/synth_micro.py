"""Time the synthetic batch renderer (synth_tiles_kernel) at the bench shape."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=384)
    ap.add_argument("--tile", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from ddlpc.data import SyntheticTiles
    ds = SyntheticTiles(100000, a.tile, classes=6, seed=3, device="cuda", layout="engine")
    idx = list(range(a.batch))
    ds.get(idx)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(a.iters):
        ds.get([j + i * a.batch for j in idx])
    e1.record()
    e1.synchronize()
    print(f"synth batch {a.batch} x {a.tile}^2: {e0.elapsed_time(e1) * 1e3 / a.iters:.1f} us per batch")


if __name__ == "__main__":
    main()
