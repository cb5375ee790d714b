"""Native build driver: compiles ``csrc/`` with hipcc for gfx950 into
``cs336_systems/_native/libcs336_hip.so`` (in-tree, so it travels to the GPU box with the repo).

No hipify, no torch.utils.cpp_extension JIT cache: kernels are plain HIP C++ for
``--offload-arch=gfx950``; the binding TU only needs the torch C++ headers (no Python headers),
since ops are registered with ``TORCH_LIBRARY``. Objects are rebuilt only when their source or
any header is newer (content-independent mtime check), compiled in parallel, then linked.

    python -m cs336_systems._native.build [--force] [-j N] [--verbose] [--save-temps]
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.dirname(os.path.abspath(__file__))
# A/B builds of kernel variants: CS336_BUILD_VARIANT=name -DFOO=1 ... builds
# _native/variants/<name>/libcs336_hip.so with those extra device defines (load it with CS336_LIB=path)
_VARIANT = os.environ.get("CS336_BUILD_VARIANT", "").split()
OBJ_DIR = os.path.join(OUT_DIR, "obj") if not _VARIANT else os.path.join(OUT_DIR, "variants", _VARIANT[0], "obj")
LIB = os.path.join(OUT_DIR, "libcs336_hip.so") if not _VARIANT else os.path.join(OUT_DIR, "variants", _VARIANT[0], "libcs336_hip.so")
EXTRA_DEFS = _VARIANT[1:]
ARCH = os.environ.get("CS336_OFFLOAD_ARCH", os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")).split(";")[0]


VGPR_FORM = ("-mllvm", "-amdgpu-mfma-vgpr-form")


def _torch_paths():
    import torch

    base = os.path.dirname(torch.__file__)
    return [os.path.join(base, "include"), os.path.join(base, "include", "torch", "csrc", "api", "include")], os.path.join(base, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _sources():
    kernels = sorted(glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True))
    # host-only TUs (torch headers): the op bindings and the hipBLASLt autotuner (csrc/blas)
    host = [os.path.join(CSRC, "bindings.cpp")] + sorted(glob.glob(os.path.join(CSRC, "blas", "*.cpp")))
    return kernels, host


def _headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _obj_for(src):
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(OBJ_DIR, rel + ".o")


def _stale(src, obj, hdr_mtime):
    if not os.path.exists(obj):
        return True
    om = os.path.getmtime(obj)
    return os.path.getmtime(src) > om or hdr_mtime > om


def build(force: bool = False, jobs: int | None = None, verbose: bool = False, save_temps: bool = False) -> str:
    incs, torch_lib, abi = _torch_paths()
    hipcc = _hipcc()
    os.makedirs(OBJ_DIR, exist_ok=True)
    kernels, host = _sources()
    hdr_mtime = max([os.path.getmtime(h) for h in _headers()] + [0])
    common = [
        "-O3",
        "-std=c++17",
        "-fPIC",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-I" + os.path.join(CSRC, "include"),
        "-I" + os.path.join(CSRC, "flash_attn"),
    ]
    # -amdgpu-mfma-vgpr-form: keep MFMA accumulators in arch VGPRs (gfx950's file is unified) instead
    # of AGPRs; otherwise hipcc copies every accumulator AGPR<->VGPR around each VALU touch
    # (online-softmax rescale), ~250 v_accvgpr moves per FA tile and half the occupancy.
    kflags = common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-Wno-unused-result", *VGPR_FORM, *EXTRA_DEFS]
    if save_temps:
        kflags += ["-save-temps=obj"]
    hflags = common + ["-DUSE_ROCM", "-D__HIP_PLATFORM_AMD__"] + ["-I" + i for i in incs] + [f"--offload-arch={ARCH}"]
    jobs_list = []
    for src in kernels:
        obj = _obj_for(src)
        if force or _stale(src, obj, hdr_mtime):
            with open(src) as fh:
                head = fh.read(4096)
            # pure-MFMA kernels (GEMM) keep accumulators in AGPRs: no VALU touches them in the loop
            agpr = "cs336-build: agpr-accumulators" in head
            flags = kflags if not agpr else [f for f in kflags if f not in VGPR_FORM]
            # MFMA loops with f32 elementwise work between the chains: keep that work scalar. The SLP
            # vectorizer packs adjacent f32 multiplies into v_pk_mul_f32, which needs register-pair
            # moves and re-aligned bf16 packing (FA2 backward dK/dV loop: 251 -> 211 VALU per 32 MFMA)
            # and is slower than two single ops beside MFMAs (MI355X_MICROARCH.md, filler prices)
            if "cs336-build: no-slp" in head:
                flags = flags + ["-fno-slp-vectorize"]
            jobs_list.append([hipcc, *flags, "-c", src, "-o", obj])
    for src in host:
        obj = _obj_for(src)
        if force or _stale(src, obj, hdr_mtime):
            jobs_list.append([hipcc, *hflags, "-x", "hip", "-c", src, "-o", obj])

    def run(cmd):
        t0 = time.time()
        r = subprocess.run(cmd, capture_output=True, text=True, cwd=OBJ_DIR)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[{time.time() - t0:5.1f}s] {os.path.basename(cmd[-3])}", flush=True)
            if r.stderr.strip():
                print(r.stderr, flush=True)
        return cmd

    if jobs_list:
        n = jobs or min(len(jobs_list), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8)
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            list(ex.map(run, jobs_list))
    objs = [_obj_for(s) for s in kernels + host]
    if force or jobs_list or not os.path.exists(LIB) or max(os.path.getmtime(o) for o in objs) > os.path.getmtime(LIB):
        tmp = LIB + ".tmp"
        cmd = [
            hipcc,
            "-shared",
            "-fPIC",
            f"--offload-arch={ARCH}",
            *objs,
            "-o",
            tmp,
            "-L" + torch_lib,
            "-lc10",
            "-lc10_hip",
            "-ltorch",
            "-ltorch_cpu",
            "-ltorch_hip",
            # torch's bundled hipBLASLt (the same library and handle torch.mm uses)
            "-lhipblaslt",
            "-Wl,-rpath," + torch_lib,
        ]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        _check_loadable(tmp)
        os.replace(tmp, LIB)
        if verbose:
            print(f"linked {LIB}", flush=True)
    return LIB


def _check_loadable(path: str) -> None:
    """dlopen the freshly linked library (RTLD_NOW): an unresolved symbol -- e.g. a kernel whose host
    stub the compiler referenced but never emitted -- fails the build here instead of on the GPU box."""
    import ctypes

    import torch  # noqa: F401  (loads libc10/libtorch the extension links against)

    try:
        ctypes.CDLL(path, mode=os.RTLD_NOW | os.RTLD_LOCAL)
    except OSError as e:
        os.remove(path)
        raise RuntimeError(f"built library does not load: {e}") from e


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--verbose", "-v", action="store_true")
    ap.add_argument("--save-temps", action="store_true")
    a = ap.parse_args(argv)
    t0 = time.time()
    path = build(a.force, a.jobs, a.verbose, a.save_temps)
    print(f"built {path} in {time.time() - t0:.1f}s (arch {ARCH}, python {sysconfig.get_python_version()})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
