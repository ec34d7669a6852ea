"""Build provenance (ops/build.py): each native library embeds the hash of the
sources and flags it was built from, the build rebuilds on an id mismatch (not on
file times), and the loader refuses a library built from other sources."""
import pytest


def test_host_library_id_matches_sources(native):
    from fastapriori_amd.ops import _native, build
    _native.host()
    got, want, path = _native.BUILD_IDS["host"]
    assert got == want == build.source_id("host") == build.embedded_id(path)


def test_source_id_tracks_content_not_mtime(tmp_path, monkeypatch):
    from fastapriori_amd.ops import build
    a = build.source_id("hip")
    assert a == build.source_id("hip") and len(a) == 16
    # other flags are another build
    assert build.source_id("hip", build.HIP_FLAGS + ["-DX"]) != a
    # the embedded id is read from the marker, without loading the file
    f = tmp_path / "lib.so"
    f.write_bytes(b"\x7fELF....FA_BUILD_ID:0123456789abcdef\x00rest")
    assert build.embedded_id(str(f)) == "0123456789abcdef"
    assert build.embedded_id(str(tmp_path / "missing.so")) is None


@pytest.mark.gpu
def test_loaded_kernel_library_was_built_from_these_sources():
    import os
    from fastapriori_amd.ops import _native, build
    assert not os.environ.get("FA_HIP_LIB")
    _native.hip()
    got, want, path = _native.BUILD_IDS["hip"]
    assert path == build.HIP_LIB
    assert got == want == build.source_id("hip") == build.embedded_id(path)
