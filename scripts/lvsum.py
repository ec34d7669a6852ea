"""Summarise bench JSON lines under gpurun_out/ (ms, levels, phase times, level plans)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "ERR", e)
        continue
    c = d["config"]
    print(f, d["ms_per_step"], c.get("levels"))
    pm = c.get("phase_ms")
    if pm:
        print("  ", {k: round(v, 1) for k, v in pm.items()})
    for k, v in (c.get("level_info") or {}).items():
        print("   ", k, {x: v[x] for x in ("kernel", "rows", "used", "sw", "cap", "passes", "pieces", "witems", "d1",
                                             "d2", "trie_reads", "slab_reads", "C", "bundled") if x in v})
