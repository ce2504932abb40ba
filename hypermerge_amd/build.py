"""Native build of the package (no cmake): hipcc for the gfx950 library,
g++ for the synthetic-feed generator.  Outputs go to hypermerge_amd/_lib/
in-tree so they travel to the GPU box with the repo snapshot."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(HERE, "_lib")
CSRC = os.path.join(HERE, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HM_OFFLOAD_ARCH", "gfx950")

GPU_SRCS = ["merge_kernels.hip", "merge_large.hip", "store_kernels.hip", "inc_kernels.hip", "exchange.hip", "cursors.hip", "engine.cpp", "store.cpp",
            "decode.cpp", "docset.cpp"]
GPU_DEPS = GPU_SRCS + ["scan.h", "merge_kernels.h", "store_kernels.h", "engine_internal.h", "../../include/hypermerge_amd.h"]


def _stale(out: str, deps) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(os.path.join(CSRC, d)) > t for d in deps)


def _run(cmd) -> None:
    print("+", " ".join(cmd), file=sys.stderr, flush=True)
    subprocess.run(cmd, check=True)


def build_gpu(force: bool = False) -> str:
    """One object per source (compiled in parallel), then one shared library."""
    out = os.path.join(LIBDIR, "libhmgpu.so")
    if force or _stale(out, GPU_DEPS):
        from concurrent.futures import ThreadPoolExecutor
        objdir = os.path.join(LIBDIR, "obj")
        os.makedirs(objdir, exist_ok=True)
        # uniform-address LDS atomics (wave ORs/mins into one word) are reduced with DPP row ops;
        # the default iterative strategy walks the active lanes on the scalar unit (~7 SALU each)
        flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                 "-mllvm", "-amdgpu-atomic-optimizer-strategy=DPP"]
        objs = [os.path.join(objdir, s + ".o") for s in GPU_SRCS]
        # plus the check build's merge_kernels object (tests only: HM_ASYNC_CHECK re-reads every
        # asynchronously loaded row set with counted loads; libhmgpu_check.so shares the other objects)
        chk_o = os.path.join(objdir, "merge_kernels_check.hip.o")
        jobs = [[HIPCC] + flags + ["-c", "-o", o, os.path.join(CSRC, src)] for src, o in zip(GPU_SRCS, objs)]
        jobs.append([HIPCC] + flags + ["-DHM_ASYNC_CHECK=1", "-c", "-o", chk_o, os.path.join(CSRC, "merge_kernels.hip")])
        with ThreadPoolExecutor(min(8, len(jobs))) as ex:
            list(ex.map(_run, jobs))
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + ["-ldl"])
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", os.path.join(LIBDIR, "libhmgpu_check.so"), chk_o] +
             [o for o in objs if not o.endswith(os.sep + "merge_kernels.hip.o")] + ["-ldl"])
    return out


def build_synth(force: bool = False) -> str:
    out = os.path.join(LIBDIR, "libhmsynth.so")
    if force or _stale(out, ["synth.cpp", "../../include/hypermerge_amd.h"]):
        os.makedirs(LIBDIR, exist_ok=True)
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-fPIC", "-shared", "-pthread", "-o", out,
              os.path.join(CSRC, "synth.cpp")])
    return out


def build_node(force: bool = False) -> str:
    """N-API addon (hypermerge_amd/js/hmgpu_node.c) over libhmgpu.so; skipped without Node headers."""
    out = os.path.join(LIBDIR, "hmgpu.node")
    src = os.path.join(HERE, "js", "hmgpu_node.c")
    if not os.path.exists("/usr/include/node/node_api.h"):
        return ""
    if force or not os.path.exists(out) or any(
            os.path.getmtime(f) > os.path.getmtime(out)
            for f in (src, os.path.join(LIBDIR, "libhmgpu.so"), os.path.join(CSRC, "../../include/hypermerge_amd.h"))):
        _run(["gcc", "-O2", "-Wall", "-shared", "-fPIC", "-I/usr/include/node",
              "-I" + os.path.join(HERE, "..", "include"), "-o", out, src, "-L" + LIBDIR, "-lhmgpu",
              "-Wl,-rpath,$ORIGIN", "-lpthread"])
    return out


def build_all(force: bool = False) -> None:
    build_gpu(force)
    build_synth(force)
    build_node(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
