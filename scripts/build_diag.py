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
    # a variant is "MODE" (conv3x3_fwd.hip with -DDDLPC_CONV_DIAG=MODE) or "unit.hip:MACRO=V[:TAG]"
    # (any unit with one macro, e.g. head_ce.hip:HEAD32_OCC=3) or "unit.hip@REV" (the unit as
    # of git revision REV: the same-box A/B baseline)
    for mode in sys.argv[1:]:
        if "@" in mode:
            unit, rev = mode.split("@")
            src = os.path.join(bdir, f"{rev}_{unit}")
            with open(src, "w") as f:
                f.write(subprocess.run(["git", "show", f"{rev}:csrc/{unit}"], cwd=be.ROOT, check=True,
                                       capture_output=True, text=True).stdout)
            defs, tag = [], f"{unit.split('.')[0]}_{rev}"
        elif ":" in mode:
            unit, macro = mode.split(":")[:2]
            src = os.path.join(be.CSRC, unit)
            defs, tag = [f"-D{macro}"], f"{unit.split('.')[0]}_{macro.replace('=', '')}"
        else:
            unit, src = "conv3x3_fwd.hip", os.path.join(be.CSRC, "conv3x3_fwd.hip")
            defs, tag = [f"-DDDLPC_CONV_DIAG={mode}"], mode
        objs = [o for o in sorted(glob.glob(os.path.join(be.BUILD, "*.o")))
                if not os.path.basename(o).startswith(unit + ".")]
        obj = os.path.join(bdir, f"{tag}.o")
        be.compile_one(src, obj, common + defs)
        lib = os.path.join(out_dir, f"libddlpc_diag_{tag}.so")
        cmd = [be.HIPCC, "-shared", "-fPIC", f"--offload-arch={be.ARCH}", "-o", lib] + objs + [obj] + [
            "-L", libdir, "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch",
            f"-Wl,-rpath,{libdir}"]
        subprocess.run(cmd, check=True)
        print(lib)


if __name__ == "__main__":
    main()
