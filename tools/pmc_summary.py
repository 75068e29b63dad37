"""Summarise a tools/profile.sh run into profiles/<tag>_*:
  <tag>_kernel_stats.csv   rocprofv3 --stats kernel table (copied)
  <tag>_kernel_stats.txt   per-kernel calls / avg us / per-step us / share
  <tag>_pmc.json           per kernel: dispatches, avg duration (trace), HBM bytes
                           per dispatch = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B; the
                           FETCH_SIZE x2 is the gfx950 correction, MI355X_MICROARCH.md)
  <tag>_bench.json         the bench line printed under the stats run
usage: python tools/pmc_summary.py gpurun_out/<tag> <tag> [out_dir (default profiles/)]

Calls per run (the divisor of every per-call figure) are the device passes the
profiled bench process made: its JSON line's `calls_made` (warmup + timed +
stage-event steps), read from each PMC run's own log, and checked against the
dispatches of the path's once-per-call marker kernel (divided by the line's
row blocks) in each PMC run and in the kernel trace.  (Before round 6 the
divisor was passed in as steps + warmup, which missed bench's untimed
stage-event steps: every round-5 per-call figure was 9/7 too high.)"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return re.sub(r"\(.*", "", name).replace("void ", "").strip()


def counters(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(list)
    if not f:
        return acc
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return acc


# a kernel each device pass dispatches once per row block, in order of preference
# (the tiled route also runs the row-merge path; the rows path on a hub block
# also computes band statistics)
MARKERS = ("k_ct_bounds", "k_rows_bin", "k_band_stats_final", "k_tcount16")


def marker_calls(dispatches, blocks):
    """(marker kernel, calls) from per-kernel dispatch counts, None if no marker ran"""
    for mk in MARKERS:
        hits = [v for k, v in dispatches.items() if k.endswith(mk)]
        if hits and hits[0]:
            return mk, hits[0] / max(1, blocks)
    return None, None


def bench_line(log):
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{\"metric\""):
                return line
    return None


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = sys.argv[3] if len(sys.argv) > 3 else os.path.join(REPO, "profiles")  # (tests: a scratch dir)
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(src, "stats", "**", "*kernel_stats.csv"), recursive=True)
    trace = glob.glob(os.path.join(src, "stats", "**", "*kernel_trace.csv"), recursive=True)
    out = {}
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
        sys.path.insert(0, os.path.join(REPO, "tools"))
        import kstats
        import io
        import contextlib
        buf = io.StringIO()
        sl0 = bench_line(os.path.join(src, "stats.log"))
        ncalls = (json.loads(sl0).get("calls_made") if sl0 else None) or 1
        with contextlib.redirect_stdout(buf):
            sys.argv = ["kstats", stats[0], str(ncalls)]  # (per_step_us = per call of the bench process)
            kstats.main()
        open(os.path.join(prof, f"{tag}_kernel_stats.txt"), "w").write(buf.getvalue())
    dur = collections.defaultdict(list)
    if trace:
        for r in csv.DictReader(open(trace[0])):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    # row-merge path: its class kernels run concurrently (4 streams); the unit the
    # bench times is the phase from the first class kernel's start to the last's
    # end in each call (a call = one k_rows_bin)
    spans, cur = [], None
    if trace:
        rows = sorted(csv.DictReader(open(trace[0])), key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            k = short(r["Kernel_Name"])
            if k.endswith("k_rows_bin"):
                if cur:
                    spans.append(cur[1] - cur[0])
                cur = None
            elif any(k.endswith(c) or c + "<" in k for c in ("k_rows_small", "k_rows_merge", "k_rows_bitmap",
                                                             "k_rows_wcount", "k_rows_wscatter", "k_rows_wunit", "k_rows_dr_prep", "k_rows_dr_fill")):
                s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                cur = [min(cur[0], s0), max(cur[1], e0)] if cur else [s0, e0]
        if cur:
            spans.append(cur[1] - cur[0])
    if spans:
        warm = sorted(spans[1:] or spans)  # (the first call also loads the kernels' code objects)
        out["_rows_phase"] = {"calls": len(spans), "median_span_us": round(warm[len(warm) // 2] / 1e3, 2),
                              "note": "first class-kernel start to last class-kernel end per call (trace), "
                                      "median over the calls after the first"}
    fetch = counters(os.path.join(src, "pmc_fetch"), "FETCH_SIZE")
    write = counters(os.path.join(src, "pmc_write"), "WRITE_SIZE")
    # calls per PMC run: what the bench process says it made, checked against the marker
    calls, check = None, {}
    for run, acc in (("pmc_fetch", fetch), ("pmc_write", write)):
        ln = bench_line(os.path.join(src, run + ".log"))
        d = json.loads(ln) if ln else {}
        blocks = int((d.get("config") or {}).get("row_blocks") or 1)
        mk, mc = marker_calls({k: len(v) for k, v in acc.items()}, blocks)
        check[run] = {"calls_made": d.get("calls_made"), "marker": mk, "marker_calls": mc, "row_blocks": blocks}
        if d.get("calls_made"):
            if calls is not None and calls != d["calls_made"]:
                raise SystemExit(f"{run}: calls_made {d['calls_made']} != the other PMC run's {calls}")
            calls = int(d["calls_made"])
        if mc is not None and d.get("calls_made") and mc != d["calls_made"]:
            raise SystemExit(f"{run}: marker {mk} says {mc} calls, bench says {d['calls_made']}")
    if trace:
        sl = bench_line(os.path.join(src, "stats.log"))
        blocks = int((json.loads(sl).get("config") or {}).get("row_blocks") or 1) if sl else 1
        mk, mc = marker_calls({k: len(v) for k, v in dur.items()}, blocks)
        check["trace"] = {"calls_made": json.loads(sl).get("calls_made") if sl else None,
                          "marker": mk, "marker_calls": mc, "row_blocks": blocks}
    tot_f = tot_w = 0.0
    for k in sorted(set(dur) | set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        out[k] = {
            "dispatches": len(dur.get(k, [])) or len(f),
            "avg_us": round(sum(dur[k]) / len(dur[k]), 2) if dur.get(k) else None,
            "fetch_bytes_per_dispatch": round(2.0 * sum(f) / len(f)) if f else None,
            "write_bytes_per_dispatch": round(sum(w) / len(w)) if w else None,
        }
        tot_f += 2.0 * sum(f)
        tot_w += sum(w)
        if f and w:
            out[k]["hbm_bytes_per_dispatch"] = out[k]["fetch_bytes_per_dispatch"] + out[k]["write_bytes_per_dispatch"]
    if calls and (tot_f or tot_w):
        # every kernel of the pass (the whole device pass), per call: the dispatches of
        # the PMC runs summed, over the calls each run makes (warmup + steps)
        out["_per_call"] = {"calls": calls, "hbm_bytes": round((tot_f + tot_w) / calls),
                            "fetch_bytes": round(tot_f / calls), "write_bytes": round(tot_w / calls),
                            "calls_check": check,
                            "note": "all kernels of one call: 2*FETCH_SIZE + WRITE_SIZE summed over the "
                                    "PMC runs' dispatches / calls per run (calls = the bench process's "
                                    "calls_made, equal to its marker kernel's dispatches / row blocks)"}
    line = bench_line(os.path.join(src, "stats.log")) or bench_line(os.path.join(src, "pmc_fetch.log"))
    if line:
        out["_workload"] = json.loads(line)["config"]["workload"]
    json.dump(out, open(os.path.join(prof, f"{tag}_pmc.json"), "w"), indent=1, sort_keys=True)
    sl = bench_line(os.path.join(src, "stats.log"))
    if sl:
        open(os.path.join(prof, f"{tag}_bench.json"), "w").write(sl)
    print(f"wrote profiles/{tag}_*")


if __name__ == "__main__":
    main()
