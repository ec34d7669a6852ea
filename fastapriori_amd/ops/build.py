"""Build the native libraries in-tree.

* ``libfa_host.so`` — C++17 host runtime (parser, Quest generator, apriori-gen,
  rules, writer, CPU reference kernels), built with g++.
* ``libfa_hip.so``  — CDNA4 kernels, built with ``hipcc --offload-arch=gfx950``.

Both are loaded through ctypes (fastapriori_amd/ops/_native.py).

Provenance: every library carries the id of what it was built from -- a hash of
its sources, headers and compile flags (``source_id``), compiled in as
``FA_BUILD_ID`` and exported as ``fa_build_id()``.  A library is rebuilt when its
embedded id differs from the id of the sources next to it (read from the file's
``FA_BUILD_ID:`` marker, without loading it), never on file times; _native checks
the id of the library it loads against the sources (the reference's Maven build is
part of its product, pom.xml:53-108).
Run ``python -m fastapriori_amd.ops.build [--force]``.
"""
from __future__ import annotations

import glob
import hashlib
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

HOST_FLAGS = ["-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", "-mpopcnt", "-fvisibility=hidden", "-Wall",
              "-Wno-unused-function"]
ASAN_FLAGS = ["-O1", "-g", "-std=c++17", "-shared", "-fPIC", "-pthread", "-mpopcnt",
              "-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
HIP_FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
             "-Wno-unused-result"]
_MARKER = b"FA_BUILD_ID:"


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libfa_hip.so)")


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def host_sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))


def hip_sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "hip", "*.hip")))


def _deps(kind: str) -> list[str]:
    if kind == "host":
        return host_sources() + sorted(glob.glob(os.path.join(CSRC, "host", "*.h")))
    return hip_sources() + sorted(glob.glob(os.path.join(CSRC, "hip", "*.h")))


def source_id(kind: str, flags: list[str] | None = None) -> str:
    """16 hex digits of sha256 over the library's sources and headers (relative path
    + bytes, sorted) and its compile flags."""
    if flags is None:
        flags = HOST_FLAGS if kind == "host" else HIP_FLAGS
    h = hashlib.sha256()
    for p in _deps(kind):
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def embedded_id(lib_path: str) -> str | None:
    """The FA_BUILD_ID a library file was built with (None: no file or no marker)."""
    try:
        with open(lib_path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(_MARKER)
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i + len(_MARKER):j].decode("ascii", "replace")


def _build(out: str, cmd_prefix: list[str], srcs: list[str], flags: list[str], bid: str) -> None:
    tmp = out + ".tmp"
    _run([*cmd_prefix, *flags, f'-DFA_BUILD_ID="{bid}"', *srcs, "-o", tmp])
    os.replace(tmp, out)


def build_host(force: bool = False, debug_sanitize: bool = False) -> str:
    out = HOST_LIB if not debug_sanitize else os.path.join(HERE, "libfa_host_asan.so")
    flags = ASAN_FLAGS if debug_sanitize else HOST_FLAGS
    bid = source_id("host", flags)
    if force or embedded_id(out) != bid:
        _build(out, ["g++"], host_sources(), flags, bid)
    return out


def build_hip(force: bool = False) -> str:
    bid = source_id("hip")
    if force or embedded_id(HIP_LIB) != bid:
        _build(HIP_LIB, [_hipcc()], hip_sources(), HIP_FLAGS, bid)
    return HIP_LIB


def build_all(force: bool = False) -> tuple[str, str]:
    return build_host(force), build_hip(force)


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build_all(force))
