"""Per-step numbers of one kernel from rocprofv3 output (dev/profiling tool).

    python tools/window_stats.py trace  RUN_kernel_trace.csv KERNEL FIRST_STEP [STEPS...]
        per-step durations of KERNEL's dispatches (the i-th dispatch = loop
        step FIRST_STEP + i) and their mean over STEPS (e.g. bench.py's
        profiled window)
    python tools/window_stats.py pmc FETCH_DIR WRITE_DIR KERNEL FIRST_STEP CONFIG N_LOCAL
        per-step HBM bytes from a FETCH_SIZE pass and a WRITE_SIZE pass
        (FETCH_SIZE KiB x 1024 x 2: the gfx950 half-count of MI355X_MICROARCH.md;
        WRITE_SIZE KiB x 1024) written into profiles/pmc_traffic.json[CONFIG]

    python tools/window_stats.py dram DIR KERNEL FIRST_STEP CONFIG N_LOCAL
        the same table from one pass of the gfx950 memory-side 32-byte
        request counters (TCC_EA0_RDREQ_DRAM_32B, TCC_EA0_WRREQ_WRITE_DRAM_32B,
        TCC_EA0_WRREQ_WRITE_ATOMIC_32B: x 32 bytes, every request width
        counted at its size - calibrated on known byte counts by
        tools/micro/fetch_calib.hip, profiles/r06_dram_counter_calibration.txt)

    python tools/window_stats.py dramstep DIR MARKER PREFIX SKIP CONFIG N_LOCAL [DOMINANT]
        the same counters summed over every kernel whose name contains PREFIX
        within each step (a step = the dispatches from one MARKER dispatch to
        the next), the first SKIP steps dropped (warmup): the mean step bytes,
        each kernel's mean bytes per dispatch, and - with DOMINANT - that
        kernel's bytes per launch as the entry's hbm_bytes_per_launch (else the
        whole step's), written into profiles/pmc_traffic.json[CONFIG]

KERNEL is a substring of the kernel name; several kernels of one step can be
given as "a+b" (their per-step values are summed, dispatches paired in order).
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dispatches(rows, kern):
    parts = kern.split("+")
    per = {p: [r for r in rows if p in r["Kernel_Name"]] for p in parts}
    n = min(len(v) for v in per.values())
    return per, n


def trace(path, kern, first, window):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    per, n = _dispatches(rows, kern)
    dur = []
    for i in range(n):
        dur.append(sum((int(per[p][i]["End_Timestamp"]) - int(per[p][i]["Start_Timestamp"])) / 1e3
                       for p in per))
    for i, v in enumerate(dur):
        print(f"step {first + i:3d} {v:9.1f} us")
    if window:
        w = [dur[s - first] for s in window if 0 <= s - first < n]
        print(f"mean over steps {window}: {sum(w) / len(w):.1f} us ({len(w)} dispatches)")


def _counter(dirpath, name, kern):
    files = glob.glob(os.path.join(dirpath, "**", "*_counter_collection.csv"), recursive=True)
    rows = [r for f in files for r in csv.DictReader(open(f)) if r["Counter_Name"] == name]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    # one row per dispatch (the counter summed over its instances)
    agg, order, names = {}, [], {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        if d not in agg:
            agg[d] = 0.0
            order.append(d)
            names[d] = r["Kernel_Name"]
        agg[d] += float(r["Counter_Value"])
    out = [{"Kernel_Name": names[d], "v": agg[d]} for d in order]
    per, n = _dispatches(out, kern)
    return [sum(per[p][i]["v"] for p in per) for i in range(n)]


def dram(ddir, kern, first, config, n_local):
    rd = [v * 32 for v in _counter(ddir, "TCC_EA0_RDREQ_DRAM_32B_sum", kern)]
    wr = [v * 32 for v in _counter(ddir, "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum", kern)]
    at = [v * 32 for v in _counter(ddir, "TCC_EA0_WRREQ_WRITE_ATOMIC_32B_sum", kern)]
    n = min(len(rd), len(wr))
    wa = [wr[i] + (at[i] if i < len(at) else 0.0) for i in range(n)]
    for i in range(n):
        print(f"step {first + i:3d}: read {rd[i] / 1e6:10.1f} MB  write {wa[i] / 1e6:8.1f} MB")
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    rec = json.load(open(path)) if os.path.exists(path) else {}
    rec[config] = {"n_local": n_local, "kernel": kern, "first_step": first,
                   "per_step_read": rd[:n], "per_step_write": wa[:n],
                   "source": f"rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum "
                             f"TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_ATOMIC_32B_sum "
                             f"({ddir}), one row per device-loop step",
                   "note": "32-byte memory-side request counts x 32 (exact for every access "
                           "width: profiles/r06_dram_counter_calibration.txt); bench.py averages "
                           "the rows of the steps it times"}
    json.dump(rec, open(path, "w"), indent=1)


def _dram_rows(dirpath):
    """{dispatch id: [kernel name, read bytes, written bytes]} from one DRAM
    counter pass (the counters summed over their instances)."""
    files = glob.glob(os.path.join(dirpath, "**", "*_counter_collection.csv"), recursive=True)
    out = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Counter_Name"]
            if name not in ("TCC_EA0_RDREQ_DRAM_32B_sum", "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum",
                            "TCC_EA0_WRREQ_WRITE_ATOMIC_32B_sum"):
                continue
            e = out.setdefault(int(r["Dispatch_Id"]), [r["Kernel_Name"], 0.0, 0.0])
            e[1 if name.startswith("TCC_EA0_RDREQ") else 2] += 32.0 * float(r["Counter_Value"])
    return out


def dramstep(ddir, marker, prefix, skip, config, n_local, dominant=None):
    rows = _dram_rows(ddir)
    ids = sorted(rows)
    marks = [i for i in ids if marker in rows[i][0]]
    steps, per_kernel = [], {}
    for a, b in zip(marks, marks[1:] + [ids[-1] + 1]):
        rd = wr = 0.0
        for i in ids:
            if a <= i < b and prefix in rows[i][0]:
                rd += rows[i][1]
                wr += rows[i][2]
                if len(steps) >= skip:
                    key = rows[i][0].replace("(anonymous namespace)::", "").split("(")[0]
                    per_kernel.setdefault(key, []).append(rows[i][1] + rows[i][2])
        steps.append((rd, wr))
    kept = steps[skip:]
    for j, (rd, wr) in enumerate(steps):
        print(f"step {j:3d}{' (skipped)' if j < skip else ''}: read {rd / 1e6:10.1f} MB  "
              f"write {wr / 1e6:8.1f} MB")
    mr = sum(r for r, _ in kept) / len(kept)
    mw = sum(w for _, w in kept) / len(kept)
    pk = {k: sum(v) / len(v) for k, v in per_kernel.items()}
    for k, v in sorted(pk.items(), key=lambda kv: -kv[1]):
        print(f"  {v / 1e6:10.1f} MB per dispatch  {k}")
    rec_path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    rec = json.load(open(rec_path)) if os.path.exists(rec_path) else {}
    dom = None
    if dominant:
        dom = [v for k, v in pk.items() if dominant in k]
        dom = dom[0] if dom else None
    rec[config] = {"n_local": n_local,
                   "kernel": dominant if dom is not None else f"all {prefix}* kernels of one step",
                   "hbm_bytes_per_launch": dom if dom is not None else mr + mw,
                   "step_bytes": mr + mw, "step_read_bytes": mr, "step_write_bytes": mw,
                   "per_kernel_bytes_per_dispatch": pk, "steps_averaged": len(kept),
                   "source": f"rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum "
                             f"TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_ATOMIC_32B_sum "
                             f"({ddir}); steps split at each {marker} dispatch, the first {skip} "
                             "dropped",
                   "note": "32-byte memory-side request counts x 32 (exact for every access "
                           "width: profiles/r06_dram_counter_calibration.txt)"}
    json.dump(rec, open(rec_path, "w"), indent=1)


def pmc(fdir, wdir, kern, first, config, n_local):
    rd = [v * 1024 * 2 for v in _counter(fdir, "FETCH_SIZE", kern)]
    wr = [v * 1024 for v in _counter(wdir, "WRITE_SIZE", kern)]
    n = min(len(rd), len(wr))
    for i in range(n):
        print(f"step {first + i:3d}: read {rd[i] / 1e6:10.1f} MB  write {wr[i] / 1e6:8.1f} MB")
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    rec = json.load(open(path)) if os.path.exists(path) else {}
    rec[config] = {"n_local": n_local, "kernel": kern, "first_step": first,
                   "per_step_read": rd[:n], "per_step_write": wr[:n],
                   "source": f"rocprofv3 --pmc FETCH_SIZE ({fdir}) and --pmc WRITE_SIZE ({wdir}), "
                             "one row per device-loop step",
                   "note": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count of wide streaming "
                           "reads, MI355X_MICROARCH.md) + WRITE_SIZE KiB x 1024; bench.py "
                           "averages the rows of the steps it times"}
    json.dump(rec, open(path, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "trace":
        trace(sys.argv[2], sys.argv[3], int(sys.argv[4]), [int(s) for s in sys.argv[5:]])
    elif sys.argv[1] == "dramstep":
        dramstep(sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]), sys.argv[6],
                 int(sys.argv[7]), sys.argv[8] if len(sys.argv) > 8 else None)
    elif sys.argv[1] == "dram":
        dram(sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5], int(sys.argv[6]))
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]), sys.argv[6], int(sys.argv[7]))
