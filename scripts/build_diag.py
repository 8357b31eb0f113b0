#!/usr/bin/env python
"""Timing-decomposition builds of the streaming 3x3 conv (never the shipped library).

    python scripts/build_diag.py 1 2 3 6 7

For each mode N, compiles csrc/conv3x3_fwd.hip with -DDDLPC_CONV_DIAG=N (1 = no fragment
LDS reads, 2 = no operand DMA, 4 = no MFMA; results are garbage) and links it with the
regular objects of build/hip into distributed-deep-learning-on-personal-computers_amd/_lib/
diag/libddlpc_diag_N.so.  Run a micro-benchmark against one with DDLPC_LIB_PATH=<that .so>.
"""
import glob
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import build_ext as be  # noqa: E402


def main():
    be.build()
    inc, libdir, abi = be.torch_paths()
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={be.ARCH}",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
              "-Wno-unused-result", "-Wno-deprecated-declarations", "-I", be.CSRC]
    for d in inc:
        common += ["-isystem", d]
    out_dir = os.path.join(be.OUT_DIR, "diag")
    bdir = os.path.join(os.path.dirname(be.BUILD), "diag")
    os.makedirs(out_dir, exist_ok=True)
    os.makedirs(bdir, exist_ok=True)
    objs = [o for o in sorted(glob.glob(os.path.join(be.BUILD, "*.o")))
            if not os.path.basename(o).startswith("conv3x3_fwd.")]
    for mode in sys.argv[1:]:
        obj = os.path.join(bdir, f"conv3x3_fwd_diag{mode}.o")
        be.compile_one(os.path.join(be.CSRC, "conv3x3_fwd.hip"), obj, common + [f"-DDDLPC_CONV_DIAG={mode}"])
        lib = os.path.join(out_dir, f"libddlpc_diag_{mode}.so")
        cmd = [be.HIPCC, "-shared", "-fPIC", f"--offload-arch={be.ARCH}", "-o", lib] + objs + [obj] + [
            "-L", libdir, "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch",
            f"-Wl,-rpath,{libdir}"]
        subprocess.run(cmd, check=True)
        print(lib)


if __name__ == "__main__":
    main()
