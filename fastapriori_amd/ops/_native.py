"""ctypes bindings for libfa_host.so (C++ runtime) and libfa_hip.so (CDNA4 kernels).

The HIP library links ``libamdhip64.so.7``; torch ships a runtime with the same
SONAME, so ``torch`` is imported (and its HIP runtime loaded) before the kernel
library is dlopen'ed — both then share one runtime and torch's streams are valid
handles for our launchers.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import build as _build

_lock = threading.Lock()
_host = None
_hip = None

i32, i64, u64, dbl = C.c_int32, C.c_int64, C.c_uint64, C.c_double
vp, cp = C.c_void_p, C.c_char_p
I64P = C.POINTER(C.c_int64)
IP = C.POINTER(C.c_int)

_HOST_SIGS = {
    "fa_parse_file": (vp, [cp, i64, i64, C.c_int, C.c_int, IP]),
    "fa_parse_buffer": (vp, [cp, i64, C.c_int, C.c_int]),
    "fa_file_size": (i64, [cp]),
    "fa_next_line_start": (i64, [cp, i64, i64]),
    "fa_chunk_scan": (None, [vp, i64, vp]),
    "fa_txndb_info": (None, [vp, vp]),
    "fa_txndb_export": (None, [vp, vp, vp, vp, C.c_int]),
    "fa_txndb_export_dict": (None, [vp, vp, vp, vp, C.c_int]),
    "fa_hash_tokens": (None, [vp, vp, i64, vp, C.c_int]),
    "fa_txndb_free": (None, [vp]),
    "fa_hash_bytes": (u64, [cp, i64]),
    "fa_quest_generate": (vp, [i64, i64, dbl, dbl, i64, i64, u64, C.c_int, C.c_int]),
    "fa_zipf_generate": (vp, [i64, i64, dbl, dbl, i64, dbl, dbl, i64, u64, C.c_int]),
    "fa_zipf_write": (C.c_int, [cp, i64, dbl, dbl, i64, dbl, dbl, i64, u64, C.c_int, C.c_int]),
    "fa_quest_write": (C.c_int, [cp, i64, dbl, dbl, i64, i64, u64, C.c_int, C.c_int]),
    "fa_apriori_gen": (vp, [vp, i64, C.c_int, C.c_int, vp]),
    "fa_cands_export": (None, [vp, vp, vp, vp]),
    "fa_cands_free": (None, [vp]),
    "fa_level_plan": (C.c_int, [vp, vp, i64, vp, vp, i32, vp, vp, i64, vp, i64, vp]),
    "fa_f1_rank_numeric": (i64, [vp, i64, i64, vp, vp, vp]),
    "fa_rules_build": (vp, [vp, vp, vp, C.c_int, vp, C.c_int, vp]),
    "fa_rules_nante": (i64, [vp]),
    "fa_rules_nstats": (i64, [vp]),
    "fa_rules_export": (None, [vp, vp, vp, vp, vp, vp]),
    "fa_rules_free": (None, [vp]),
    "fa_recommend_cpu": (None, [vp, vp, vp, i64, i32, vp, vp, i64, vp, C.c_int]),
    "fa_write_freq_itemsets": (C.c_int, [cp, vp, vp, i32, vp, vp, vp, C.c_int, C.c_int, C.c_int]),
    "fa_cpu_histogram": (None, [vp, i64, i64, vp, C.c_int]),
    "fa_build_probe_table": (None, [vp, i64, C.c_int, C.c_uint32, vp, vp]),
    "fa_cpu_txn_freq_count": (None, [vp, vp, i64, vp, vp, C.c_int]),
    "fa_cpu_compress": (None, [vp, vp, vp, vp, i64, vp, vp, C.c_int]),
    "fa_cpu_build_bitmaps": (None, [vp, vp, vp, i64, i64, vp, C.c_int]),
    "fa_cpu_row_hash": (None, [vp, vp, i64, vp, vp, C.c_int]),
    "fa_cpu_pair_gram": (None, [vp, i32, i64, i64, vp, vp, C.c_int]),
    "fa_cpu_pair_horizontal": (None, [vp, vp, i64, vp, i32, vp, C.c_int]),
    "fa_cpu_count_candidates": (None, [vp, i64, i64, vp, i32, vp, vp, i64, vp, vp, C.c_int]),
}

_HIP_SIGS = {
    "fa_hip_histogram": (C.c_int, [vp, i64, i32, vp, vp]),
    "fa_hip_f1_rank": (C.c_int, [vp, i32, i64, C.c_int, vp, vp, vp]),
    "fa_hip_debug_la_qsum": (C.c_int, [vp, vp]),
    "fa_hip_win_alive": (C.c_int, [vp, i64, vp, C.c_int, i64, C.c_int, vp, vp, vp]),
    "fa_hip_win_compact": (C.c_int, [vp, i64, vp, C.c_int, i64, vp, vp, vp, i64, vp]),
    "fa_hip_debug_slab_max_wg": (None, [C.c_int]),
    "fa_hip_pairs_compact": (C.c_int, [vp, i64, i32, i64, vp, vp, vp, vp, vp, vp]),
    "fa_hip_f1_sketch": (C.c_int, [vp, i64, vp, vp, vp]),
    "fa_hip_f1_exact": (C.c_int, [vp, i64, vp, C.c_int, vp, vp]),
    "fa_hip_txn_freq_count": (C.c_int, [vp, vp, i64, i64, vp, vp, vp]),
    "fa_hip_compress_regs": (C.c_int, [C.c_int, vp, vp, vp, vp, i64, vp, vp, vp, vp, vp]),
    "fa_hip_ag_gen": (C.c_int, [vp, i64, C.c_int, C.c_int, vp, i64, vp, i64, vp, vp]),
    "fa_hip_ag_chain": (C.c_int, [vp, i64, C.c_int, C.c_int, vp, i64, vp, i64, C.c_int, dbl, i64, i64, vp, vp,
                                  C.c_int, dbl]),
    "fa_hip_ag_build": (C.c_int, [vp, i64, C.c_int, vp, C.c_uint32, C.c_int, vp, vp]),
    "fa_hip_ag_rows": (C.c_int, [vp, i64, C.c_int, vp, C.c_uint32, C.c_int, vp, vp, vp, vp, C.c_int, vp]),
    "fa_hip_cmp_agg": (C.c_int, [vp, vp, vp, i64, vp, vp, vp, C.c_int, vp]),
    "fa_hip_cmp_scan": (C.c_int, [vp, vp, i64, C.c_int, vp, vp, vp, vp, vp]),
    "fa_hip_cmp_emit": (C.c_int, [vp, vp, vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, C.c_int, vp, vp, i64, vp, vp,
                                  vp]),
    "fa_hip_lr_rows": (C.c_int, [vp, vp, vp, i64, vp, C.c_int, vp, i64, vp]),
    "fa_hip_compress_regs_bc": (C.c_int, [vp, vp, vp, vp, i64, vp, vp, vp, vp, vp, i64, C.c_int, vp]),
    "fa_hip_block_counts_rows": (C.c_int, [vp, vp, vp, i64, vp, i64, C.c_int, vp, vp]),
    "fa_hip_block_bsum": (C.c_int, [vp, i64, i64, C.c_int, vp, vp]),
    "fa_hip_compress_staged": (C.c_int, [vp, vp, vp, i64, vp, vp, vp, vp, vp]),
    "fa_hip_compress_staged64": (C.c_int, [vp, vp, vp, i64, vp, vp, vp, vp, C.c_int, vp]),
    "fa_hip_count_slab_rec": (C.c_int, [vp, vp, vp, i64, vp, C.c_int, C.c_int, vp, vp, C.c_int, C.c_int, vp, vp,
                                        C.c_int, C.c_int, vp, i64, vp, vp, vp]),
    "fa_hip_count_slab_rec_cls": (C.c_int, [vp, vp, vp, i64, vp, C.c_int, C.c_int, vp, vp, C.c_int, C.c_int, vp,
                                            vp, C.c_int, C.c_int, vp, i64, vp, vp, vp, C.c_int]),
    # device-resident level bundles (gen.hip fa_hip_dl_*, levels.hip)
    "fa_hip_dl_level0": (C.c_int, [vp, vp, i64, i64, C.c_int, C.c_int, vp, i64, vp, vp, i64, dbl, dbl, vp, C.c_int,
                                   vp]),
    "fa_hip_dl_more": (C.c_int, [C.c_int, vp, i64, i64, vp, vp, dbl, C.c_int, dbl, dbl, i64, vp, vp, vp, vp]),
    "fa_hip_dl_plan": (C.c_int, [vp, C.c_int, vp, C.c_int, vp, vp, i64, vp, i64, vp, i64, C.c_int, vp]),
    "fa_hip_set_lane_deal": (None, [C.c_int]),
    "fa_hip_set_cap_max": (None, [C.c_int]),
    "fa_hip_set_piece_part": (C.c_int, [C.c_int, C.c_int]),
    "fa_hip_dl_gpre_need": (i64, [vp, C.c_int]),
    "fa_hip_dl_plan_window": (C.c_int, [vp, C.c_int, vp, C.c_int, vp, vp, i64, vp, i64, vp, i64, i64, i64, C.c_int,
                                        vp]),
    "fa_hip_dl_plan_window_bits": (C.c_int, [vp, C.c_int, vp, C.c_int, vp, vp, vp, i64, vp, i64, vp, i64, i64, i64,
                                             C.c_int, vp]),
    "fa_hip_dl_chunk_bits": (C.c_int, [vp, C.c_int, C.c_int, vp, vp]),
    "fa_hip_dl_threshold": (C.c_int, [vp, C.c_int, vp, i64, vp, vp, vp, vp, vp, vp, i64, vp]),
    "fa_hip_trim_scan_count": (C.c_int, [vp, vp, i64, vp, C.c_int, C.c_int, vp, vp, vp, vp, vp]),
    "fa_hip_trim_emit": (C.c_int, [vp, vp, vp, C.c_int, i64, vp, vp, vp, vp, vp, vp, vp, vp]),
    "fa_hip_compress_wave": (C.c_int, [vp, vp, vp, vp, i64, vp, vp, vp, C.c_int, vp, vp]),
    "fa_hip_compress_lds": (C.c_int, [vp, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp]),
    "fa_hip_dedup_probe": (C.c_int, [vp, vp, vp, i64, vp, vp, vp]),
    "fa_hip_row_hash": (C.c_int, [vp, vp, i64, vp, vp, vp]),
    "fa_hip_build_bitmaps": (C.c_int, [vp, vp, vp, i64, i32, i64, C.c_int, C.c_int, vp, vp, vp, C.c_int, vp]),
    "fa_hip_block_counts": (C.c_int, [vp, vp, i64, i32, vp, vp, C.c_int, vp]),
    "fa_hip_block_scatter": (C.c_int, [vp, vp, i64, i32, vp, vp, vp, C.c_int, vp]),
    "fa_hip_pair_queue16": (C.c_int, [vp, vp, vp, i64, C.c_int, i64, vp, vp, C.c_int, vp]),
    "fa_hip_pair_blocked": (C.c_int, [vp, vp, vp, i64, vp, i32, vp, i64, vp]),
    "fa_hip_pair_gram_mfma": (C.c_int, [vp, i32, i64, i64, C.c_int, i64, vp, C.c_int, C.c_uint32, C.c_int, vp]),
    "fa_hip_pair_gram_popc": (C.c_int, [vp, i32, i64, i64, C.c_int, i64, vp, vp, C.c_int, vp]),
    "fa_hip_count_candidates": (C.c_int, [vp, i64, i64, vp, C.c_int, vp, vp, vp, C.c_int, vp, vp, vp]),
    "fa_hip_recommend": (C.c_int, [vp, vp, vp, i64, i32, vp, vp, i64, vp, vp]),
    "fa_hip_recommend_indexed": (C.c_int, [vp, vp, vp, vp, vp, i64, i32, vp, vp, i64, vp, vp]),
    "fa_hip_parse_tiles": (i64, [i64]),
    "fa_hip_tparse_tiles": (i64, [i64, i64]),
    "fa_hip_tparse_hist_cap": (C.c_int, []),
    "fa_hip_tline_count": (C.c_int, [vp, i64, i64, vp, vp]),
    "fa_hip_tparse": (C.c_int, [vp, i64, i64, i64, C.c_int, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "fa_hip_scan_small": (C.c_int, [C.c_int, vp, i64, vp, vp, vp]),
    "fa_hip_tcompact": (C.c_int, [vp, vp, i64, C.c_int, vp, vp, vp, vp, vp, vp, vp, i64, vp, C.c_int, vp, vp, vp]),
    "fa_hip_hist_reduce": (C.c_int, [vp, C.c_int, vp, vp]),
    "fa_hip_line_count": (C.c_int, [vp, i64, vp, vp]),
    "fa_hip_line_ends": (C.c_int, [vp, i64, vp, vp, vp]),
    "fa_hip_parse_lines_dict": (C.c_int, [vp, vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, vp]),
    "fa_hip_slot_remap": (C.c_int, [vp, i64, vp, vp]),
    "fa_hip_dict_verify": (C.c_int, [vp, vp, i64, vp, vp, vp, vp, i64, vp]),
    "fa_hip_compact_lines": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, vp, vp, vp]),
    "fa_hip_rule_gen": (C.c_int, [vp, i64, C.c_int, vp, i64, vp, vp, vp, vp, vp]),
    "fa_hip_rule_cut": (C.c_int, [vp, vp, i64, C.c_int, vp, vp, vp, vp]),
    "fa_hip_rule_emit": (C.c_int, [vp, vp, vp, vp, vp, i64, vp, vp]),
}


def _declare(lib, sigs):
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


BUILD_IDS: dict = {}     # loaded library -> (embedded FA_BUILD_ID, id of the sources next to it)


def _check_id(kind: str, lib, path: str) -> None:
    """The loaded library must have been built from the sources in this tree
    (ops/build.py source_id): a stale or foreign build fails loudly instead of
    running code the tree does not hold.  FA_HIP_LIB (another build for A/B runs)
    and a tree without sources (an installed copy) are recorded, not checked."""
    fn = lib.fa_build_id
    fn.restype, fn.argtypes = cp, []
    got = fn().decode("ascii", "replace")
    have_src = bool(_build.hip_sources() if kind == "hip" else _build.host_sources())
    want = _build.source_id(kind) if have_src else None
    BUILD_IDS[kind] = (got, want, path)
    override = kind == "hip" and bool(os.environ.get("FA_HIP_LIB"))
    if want is not None and got != want and not override:
        raise RuntimeError(f"{path} was built from other sources (build id {got}, these sources {want}): "
                           "rebuild with `python -m fastapriori_amd.ops.build`")


def host():
    global _host
    if _host is None:
        with _lock:
            if _host is None:
                path = _build.HOST_LIB
                if _build.embedded_id(path) != _build.source_id("host") and _build.host_sources():
                    _build.build_host()
                lib = C.CDLL(path)
                _check_id("host", lib, path)
                _host = _declare(lib, _HOST_SIGS)
    return _host


def hip():
    """The kernel library.  Raises loudly when it is missing: there is no fallback."""
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                import torch  # noqa: F401  (load torch's HIP runtime first; see module doc)
                # FA_HIP_LIB: another build of the same sources' ABI (A/B runs of kernel variants)
                path = os.environ.get("FA_HIP_LIB") or _build.HIP_LIB
                if not os.path.exists(path):
                    raise RuntimeError(
                        f"{path} is missing: build it with `python -m fastapriori_amd.ops.build` "
                        "(the GPU path has no non-native fallback)")
                lib = C.CDLL(path)
                _check_id("hip", lib, path)
                _hip = _declare(lib, _HIP_SIGS)
    return _hip


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error code {rc}")
