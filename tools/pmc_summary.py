"""Summarise the rocprofv3 --pmc passes of tools/pmc_lloyd.sh (per dispatch).

    python tools/pmc_summary.py gpurun_out/pmc_c3 > profiles/rNN_pmc_screen32.txt
    python tools/pmc_summary.py gpurun_out/pmc_c3 --json 3 100000000   # -> profiles/pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes
of wide coalesced streaming reads (MI355X_MICROARCH.md §HBM), so the HBM read
bytes reported below are FETCH_SIZE * 1024 * 2.
"""
import collections
import csv
import glob
import os
import sys

roots = [a for a in sys.argv[1:] if not a.startswith("--") and os.path.isdir(a)] or ["gpurun_out/pmc"]
root = roots[0]
json_cfg = None
want_arg = None
if "--want" in sys.argv:
    want_arg = sys.argv[sys.argv.index("--want") + 1].split(",")
if "--json" in sys.argv:
    i = sys.argv.index("--json")
    json_cfg, json_n = sys.argv[i + 1], int(sys.argv[i + 2])
agg = collections.defaultdict(dict)
names = {}
files = [f for r0 in roots for f in sorted(glob.glob(os.path.join(r0, "*", "*_counter_collection.csv")) + glob.glob(os.path.join(r0, "*_counter_collection.csv")))]
for f in files:
    for r in csv.DictReader(open(f)):
        # passes of one command line pair up by dispatch id (same launch order)
        key = ("+".join(os.path.basename(r0) for r0 in roots), int(r["Dispatch_Id"]))
        names[key] = r["Kernel_Name"]
        agg[key][r["Counter_Name"]] = agg[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
want = tuple(want_arg) if want_arg else ("screen32", "fallback32", "reduce32", "screen_fast",
                                         "screen_kernel")
for key in sorted(agg):
    nm = names[key]
    if not any(w in nm for w in want):
        continue
    c = agg[key]
    line = f"{key[0]} dispatch {key[1]:4d} {nm[:70]}\n   "
    line += " ".join(f"{k}={v:.6g}" for k, v in sorted(c.items()))
    if "FETCH_SIZE" in c:
        line += f"\n   HBM read bytes = FETCH_SIZE*1024*2 = {c['FETCH_SIZE'] * 2048:.4g}"
    if "WRITE_SIZE" in c:
        line += f"\n   HBM write bytes = WRITE_SIZE*1024 = {c['WRITE_SIZE'] * 1024:.4g}"
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        w = c["SQ_WAVE_CYCLES"]
        line += (f"\n   wave-cycle split: active {c.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f}"
                 f" issue-stall {c.get('SQ_WAIT_INST_ANY', 0) / w:.2f}"
                 f" waitcnt {c.get('SQ_WAIT_ANY', 0) / w:.2f}")
    print(line)

if json_cfg is not None and "--groupby" in sys.argv:
    # config 4: HBM bytes of all group-by kernels (gb_*) of one step = their
    # total over the run / the number of gb_hist1 launches (one per step)
    import json
    steps = sum(1 for k in agg if "gb_hist1" in names[k] and "FETCH_SIZE" in agg[k])
    # gb_tsr_*: the producer's timestamp range, once per event set, not per step
    step_k = [k for k in agg if "gb_" in names[k] and "gb_tsr" not in names[k]]
    rb = sum(agg[k]["FETCH_SIZE"] for k in step_k if "FETCH_SIZE" in agg[k]) * 2048
    wb = sum(agg[k]["WRITE_SIZE"] for k in step_k if "WRITE_SIZE" in agg[k]) * 1024
    if steps:
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "profiles", "pmc_traffic.json")
        rec = json.load(open(path)) if os.path.exists(path) else {}
        rec[json_cfg] = {"n_local": json_n, "hbm_bytes_per_launch": (rb + wb) / steps,
                         "read_bytes": rb / steps, "write_bytes": wb / steps, "source": root,
                         "kernel": "all gb_* kernels of one group-by step",
                         "note": "FETCH_SIZE KiB x2 (gfx950 half-count) + WRITE_SIZE KiB, "
                                 "summed over the step's kernels"}
        json.dump(rec, open(path, "w"), indent=1)
        print("wrote", path, rec[json_cfg])
    json_cfg = None

if json_cfg is not None:
    # HBM bytes of the last steady-state (DELTA) screen32 launch: read + write
    import json
    f = [k for k in agg if "screen32" in names[k] and "FETCH_SIZE" in agg[k]]
    w = [k for k in agg if "screen32" in names[k] and "WRITE_SIZE" in agg[k]]
    if f and w:
        rb = agg[max(f, key=lambda k: k[1])]["FETCH_SIZE"] * 2048
        wb = agg[max(w, key=lambda k: k[1])]["WRITE_SIZE"] * 1024
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "profiles", "pmc_traffic.json")
        rec = json.load(open(path)) if os.path.exists(path) else {}
        rec[json_cfg] = {"n_local": json_n, "hbm_bytes_per_launch": rb + wb, "read_bytes": rb,
                         "write_bytes": wb, "source": root,
                         "kernel": names[max(f, key=lambda k: k[1])],
                         "note": "FETCH_SIZE KiB x2 (gfx950 half-count) + WRITE_SIZE KiB"}
        json.dump(rec, open(path, "w"), indent=1)
        print("wrote", path, rec[json_cfg])
