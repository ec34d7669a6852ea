"""Build the native libraries in-tree.

* ``libfa_host.so`` — C++17 host runtime (parser, Quest generator, apriori-gen,
  rules, writer, CPU reference kernels), built with g++.
* ``libfa_hip.so``  — CDNA4 kernels, built with ``hipcc --offload-arch=gfx950``.

Both are loaded through ctypes (fastapriori_amd/ops/_native.py).  The build is
incremental: a library is rebuilt only when a source or header is newer.
Run ``python -m fastapriori_amd.ops.build [--force]``.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "csrc")
HOST_LIB = os.path.join(HERE, "libfa_host.so")
HIP_LIB = os.path.join(HERE, "libfa_hip.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libfa_hip.so)")


def _stale(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def host_sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))


def hip_sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "hip", "*.hip")))


def build_host(force: bool = False, debug_sanitize: bool = False) -> str:
    srcs = host_sources()
    deps = srcs + glob.glob(os.path.join(CSRC, "host", "*.h"))
    out = HOST_LIB if not debug_sanitize else os.path.join(HERE, "libfa_host_asan.so")
    if force or _stale(out, deps):
        flags = ["-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", "-mpopcnt",
                 "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]
        if debug_sanitize:
            flags = ["-O1", "-g", "-std=c++17", "-shared", "-fPIC", "-pthread", "-mpopcnt",
                     "-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
        tmp = out + ".tmp"
        _run(["g++", *flags, *srcs, "-o", tmp])
        os.replace(tmp, out)
    return out


def build_hip(force: bool = False) -> str:
    srcs = hip_sources()
    deps = srcs + glob.glob(os.path.join(CSRC, "hip", "*.h"))
    if force or _stale(HIP_LIB, deps):
        tmp = HIP_LIB + ".tmp"
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
              "-fvisibility=hidden", "-Wno-unused-result", *srcs, "-o", tmp])
        os.replace(tmp, HIP_LIB)
    return HIP_LIB


def build_all(force: bool = False) -> tuple[str, str]:
    return build_host(force), build_hip(force)


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build_all(force))
