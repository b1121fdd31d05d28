"""In-tree build of the native runtime (``_C``) for gfx950.

Drives ``hipcc`` directly through a generated ninja file (no hipify step, no JIT cache): the HIP
kernels under ``csrc/kernels`` are plain HIP compiled for ``--offload-arch=gfx950``; the runtime
under ``csrc/runtime`` (torch op wrappers, RCCL communicator, bucketed reducer, pybind module) is
host C++ compiled against the installed PyTorch-ROCm headers. The resulting
``_C.cpython-*.so`` lands next to this file so it travels with the repository snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD_DIR = os.path.join(REPO, "build", "native")
ARCH = os.environ.get("CDP_OFFLOAD_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
OUTPUT = os.path.join(PKG_DIR, "_C" + EXT_SUFFIX)

KERNELS = ["conv_igemm.hip", "conv_x3.hip", "wgrad.hip", "bn.hip", "misc.hip", "stem.hip", "bwd_fuse.hip", "bwd_pair.hip",
           "bwd_pair_d128x128.hip", "bwd_pair_d128x64.hip", "bwd_pair_d64x128.hip", "bwd_pair_d64x64.hip"]
RUNTIME = ["ops.cpp", "rccl_comm.cpp", "reducer.cpp", "torch_ops.cpp", "bindings.cpp"]


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build the native runtime)")


# GEMM kernels whose operand split must stay scalar f32: packed-f32 VALU issued between MFMAs
# costs ~22 extra cycles per MFMA gap on gfx950 (x3_common.h), and the SLP vectorizer would re-pack
# adjacent scalar multiplies / FMAs into v_pk_mul_f32 / v_pk_fma_f32
NO_SLP = {"conv_x3.hip", "wgrad.hip", "bwd_pair.hip", "bwd_pair_d128x128.hip", "bwd_pair_d128x64.hip",
          "bwd_pair_d64x128.hip", "bwd_pair_d64x64.hip"}


def _ninja_escape(s: str) -> str:
    return s.replace("$", "$$").replace(" ", "$ ").replace(":", "$:")


def write_ninja() -> str:
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    hipcc = _hipcc()
    os.makedirs(BUILD_DIR, exist_ok=True)
    kflags = f"--offload-arch={ARCH} -O3 -fPIC -std=c++17 -ffp-contract=fast -Wno-unused-result"
    if os.environ.get("CDP_KFLAGS_EXTRA"):  # extra kernel flags for A/B builds (e.g. -DCDP_INTERLEAVE_VPM=2)
        kflags += " " + os.environ["CDP_KFLAGS_EXTRA"]
    rflags = " ".join(
        [
            f"--offload-arch={ARCH} -O2 -fPIC -std=c++17 -w",
            "-D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DUSE_DISTRIBUTED -DUSE_C10D_GLOO",
            "-DTORCH_EXTENSION_NAME=_C -DTORCH_API_INCLUDE_EXTENSION_H",
            f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        ]
        + [f"-I{p}" for p in inc + [py_inc, "/opt/rocm/include"]]
    )
    ldflags = " ".join(
        [
            "-shared -fPIC",
            f"-L{lib}",
            "-lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -lrccl",
            "-L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib",
            f"-Wl,-rpath,{lib}",
        ]
    )
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"kflags = {kflags}",
        f"rflags = {rflags}",
        f"ldflags = {ldflags}",
        "rule kcc",
        "  command = $hipcc $kflags $kextra -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC(gfx950) $in",
        "rule rcc",
        "  command = $hipcc $rflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link",
        "  command = $hipcc $in $ldflags -o $out",
        "  description = LINK $out",
    ]
    objs = []
    for f in KERNELS:
        src = os.path.join(CSRC, "kernels", f)
        obj = os.path.join(BUILD_DIR, f + ".o")
        lines.append(f"build {_ninja_escape(obj)}: kcc {_ninja_escape(src)}")
        if f in NO_SLP:
            lines.append("  kextra = -fno-slp-vectorize")
        objs.append(obj)
    for f in RUNTIME:
        src = os.path.join(CSRC, "runtime", f)
        obj = os.path.join(BUILD_DIR, f + ".o")
        lines.append(f"build {_ninja_escape(obj)}: rcc {_ninja_escape(src)}")
        objs.append(obj)
    lines.append(f"build {_ninja_escape(OUTPUT)}: link " + " ".join(_ninja_escape(o) for o in objs))
    lines.append(f"default {_ninja_escape(OUTPUT)}")
    path = os.path.join(BUILD_DIR, "build.ninja")
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    return path


def build(verbose: bool = False, jobs: int | None = None) -> str:
    """Compile (incrementally) and return the path of the built extension."""
    ninja_file = write_ninja()
    ninja = shutil.which("ninja")
    if ninja is None:
        raise RuntimeError("ninja not found")
    if jobs is None:
        jobs = min(8, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)))
    cmd = [ninja, "-f", ninja_file, "-j", str(jobs)]
    if verbose:
        cmd.append("-v")
    res = subprocess.run(cmd, cwd=BUILD_DIR, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout)
        raise RuntimeError("native build failed")
    if verbose:
        sys.stdout.write(res.stdout)
    return OUTPUT


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
