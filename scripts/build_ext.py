#!/usr/bin/env python
"""Build the gfx950 HIP kernel library in-tree: csrc/*.hip + bindings.cpp -> ddlpc/_lib/libddlpc_hip.so

Plain hipcc (no hipify, no JIT cache): every translation unit is compiled with
``--offload-arch=gfx950`` in parallel, then linked against the libtorch that ships with
the installed PyTorch (its bundled HIP runtime is reused at load time: same soname).
Incremental: a unit is rebuilt when it or any csrc header is newer than its object.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "distributed-deep-learning-on-personal-computers_amd")
OUT_DIR = os.path.join(PKG, "_lib")
BUILD = os.path.join(ROOT, "build", "hip")
LIB = os.path.join(OUT_DIR, "libddlpc_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def torch_paths():
    import torch
    from torch.utils import cpp_extension
    inc = cpp_extension.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def compile_one(src, obj, flags):
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(verbose=False, jobs=None, force=False):
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(BUILD, exist_ok=True)
    inc, libdir, abi = torch_paths()
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
              "-Wno-unused-result", "-Wno-deprecated-declarations", "-I", CSRC]
    for d in inc:
        common += ["-isystem", d]
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    hdr_mtime = max((os.path.getmtime(h) for h in headers), default=0)
    # bindings.cpp: host code with HIP launches; cpu_ref.cpp: the CPU kernels (plain C++)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip"))) + [os.path.join(CSRC, "bindings.cpp"),
                                                             os.path.join(CSRC, "cpu_ref.cpp")]
    todo, objs = [], []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if force or not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_mtime):
            flags = list(common)
            if s.endswith("cpu_ref.cpp"):
                flags = ["-x", "c++"] + [f for f in flags if not f.startswith("--offload-arch")]
            elif s.endswith(".cpp"):
                flags = ["-x", "hip"] + flags
            todo.append((s, o, flags))
    jobs = jobs or min(len(todo) or 1, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(compile_one, *t) for t in todo]
            for f in cf.as_completed(futs):
                o, err = f.result()
                if verbose:
                    print("built", os.path.basename(o), file=sys.stderr)
                    if err.strip():
                        print(err, file=sys.stderr)
    need_link = bool(todo) or not os.path.exists(LIB) or \
        os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs)
    if need_link:
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs + [
            "-L", libdir, "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch",
            f"-Wl,-rpath,{libdir}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(a.verbose, a.jobs, a.force))
