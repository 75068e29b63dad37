"""Summarise a tools/profile.sh run into profiles/<tag>_*:
  <tag>_kernel_stats.csv   rocprofv3 --stats kernel table (copied)
  <tag>_kernel_stats.txt   per-kernel calls / avg us / per-step us / share
  <tag>_pmc.json           per kernel: dispatches, avg duration (trace), HBM bytes
                           per dispatch = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B; the
                           FETCH_SIZE x2 is the gfx950 correction, MI355X_MICROARCH.md)
  <tag>_bench.json         the bench line printed under the stats run
usage: python tools/pmc_summary.py gpurun_out/<tag> <tag> <dispatches_per_kernel_per_run>"""
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


def bench_line(log):
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{\"metric\""):
                return line
    return None


def main():
    src, tag = sys.argv[1], sys.argv[2]
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # (read before kstats rewrites sys.argv)
    prof = os.path.join(REPO, "profiles")
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
        with contextlib.redirect_stdout(buf):
            sys.argv = ["kstats", stats[0]]
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
                                                             "k_rows_wcount", "k_rows_wscatter", "k_rows_wunit", "k_rows_wgather", "k_rows_dr_prep", "k_rows_dr_fill")):
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
                            "note": "all kernels of one call: 2*FETCH_SIZE + WRITE_SIZE summed over the "
                                    "PMC runs' dispatches / calls per run"}
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
