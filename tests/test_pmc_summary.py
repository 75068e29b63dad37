"""tools/pmc_summary.py's per-call accounting (CPU): the divisor of every
per-call byte figure is the device passes the profiled bench process made
(its JSON line's calls_made), which must agree with the once-per-call marker
kernel's dispatches.  Round 5 divided by steps + warmup (7) while bench made
9 calls (two untimed stage-event steps), overstating every figure by 9/7."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"tsg::k_rows_bin": (1000.0, 500.0), "tsg::k_rows_compact": (64000.0, 32000.0),
           "void tsg::k_rows_merge<64, 256, 62>": (8000.0, 4000.0)}  # (FETCH_SIZE, WRITE_SIZE) in KiB


def _write_run(d, counter, idx, calls, blocks):
    os.makedirs(os.path.join(d, "run"), exist_ok=True)
    with open(os.path.join(d, "run", "x_counter_collection.csv"), "w") as f:
        f.write("Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n")
        i = 0
        for _ in range(calls * blocks):
            for k, v in KERNELS.items():
                i += 1
                f.write(f'{i},"{k}(RowsArgs)",{counter},{v[idx]}\n')


def _line(calls, blocks):
    return json.dumps({"metric": "m", "calls_made": calls, "config": {"workload": "w", "row_blocks": blocks}})


def _run(tmp_path, calls, blocks, made=None):
    src = tmp_path / "src"
    for run, counter, idx in (("pmc_fetch", "FETCH_SIZE", 0), ("pmc_write", "WRITE_SIZE", 1)):
        _write_run(str(src / run), counter, idx, calls, blocks)
        (src / (run + ".log")).write_text("noise\n" + _line(made or calls, blocks) + "\n")
    out = tmp_path / "out"
    return subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), str(src), "t", str(out)],
                          capture_output=True, text=True), out


def test_nine_dispatches_over_nine_calls_is_one_dispatch_per_call(tmp_path):
    r, out = _run(tmp_path, calls=9, blocks=1)
    assert r.returncode == 0, r.stderr
    d = json.load(open(out / "t_pmc.json"))
    pc = d["_per_call"]
    assert pc["calls"] == 9
    one = sum(2.0 * f * 1024 + w * 1024 for f, w in KERNELS.values())  # one dispatch of each kernel
    assert pc["hbm_bytes"] == round(one)
    assert pc["calls_check"]["pmc_fetch"]["marker"] == "k_rows_bin"
    assert pc["calls_check"]["pmc_fetch"]["marker_calls"] == 9
    k = d["tsg::k_rows_compact"]
    assert k["dispatches"] == 9 and k["hbm_bytes_per_dispatch"] == round(2 * 64000.0 * 1024 + 32000.0 * 1024)


def test_row_blocks_divide_the_marker(tmp_path):
    # sequential row blocks (LiveJournal): the marker runs once per block per call
    r, out = _run(tmp_path, calls=4, blocks=90)
    assert r.returncode == 0, r.stderr
    pc = json.load(open(out / "t_pmc.json"))["_per_call"]
    assert pc["calls"] == 4 and pc["calls_check"]["pmc_write"]["marker_calls"] == 4
    one = sum(2.0 * f * 1024 + w * 1024 for f, w in KERNELS.values())
    assert pc["hbm_bytes"] == round(90 * one)


def test_disagreeing_call_counts_fail_loudly(tmp_path):
    r, _ = _run(tmp_path, calls=9, blocks=1, made=7)
    assert r.returncode != 0 and "marker" in (r.stderr + r.stdout)


def test_bench_pmc_traffic_counts_dispatches_per_call(tmp_path):
    sys.path.insert(0, REPO)
    import bench
    p = tmp_path / "p.json"
    p.write_text(json.dumps({"_per_call": {"calls": 9, "hbm_bytes": 123},
                             "tsg::k_rows_wunit": {"dispatches": 810, "hbm_bytes_per_dispatch": 1000},
                             "tsg::k_rows_merge": {"dispatches": 9, "hbm_bytes_per_dispatch": 10}}))
    unit, allk = bench.pmc_traffic(["k_rows_wunit", "k_rows_merge"], str(p))
    assert unit == 90 * 1000 + 10 and allk == 123


def test_newest_profile_by_round_and_tag_order(tmp_path):
    """bench.pmc_file's default: the newest summary of the workload by round,
    then by tag in the order tags are handed out (x < aa < bf), not by name."""
    import json
    import bench
    (tmp_path / "profiles").mkdir()
    for tag in ("r5z", "r6x", "r6aa", "r6bf", "r6c"):
        (tmp_path / "profiles" / f"{tag}_webbase_pmc.json").write_text(json.dumps({"_workload": "w"}))
    (tmp_path / "profiles" / "r6zz_other_pmc.json").write_text(json.dumps({"_workload": "other"}))
    got = bench.pmc_file("w", root=str(tmp_path))
    assert os.path.basename(got) == "r6bf_webbase_pmc.json"
