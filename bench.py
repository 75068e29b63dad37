"""bench.py -- TileSpGEMM on MI355X: SpGEMM GFLOPS (fp64, C = A^2) + HBM roofline.

One "step" = one full device pass of the hot path on one matrix, device CSR in ->
device CSR out: GPU csr2tile(A) + csr2tile(B) + step 1 + step 2 (+ scan) +
step 3 + GPU tile2csr (SURVEY.md §8d t_e2e).  Inputs are resident in HBM
(torch tensors) before the timed region.  GFLOPS = 2*nnzCub/t
(src/tilespgemm-cuda.h:2808).

  python bench.py                       # N=1, webbase-1M synthetic stand-in
  python bench.py --gpus N ...          # under torch.distributed.run (default: strong
                                        # scaling, north_star's exchange): the fixed
                                        # product A*B, A's rows split into pieces of
                                        # equal work, B replicated, C gathered to rank 0
                                        # over RCCL inside the timed region (gather_ms
                                        # reported; gather-bound: DESIGN 5)
  python bench.py --gpus N --scaling weak
                                        # NOT the north-star metric: rank r computes row
                                        # block r of [A; A; ...; A]*B (one full A per
                                        # rank, B replicated, C stays distributed, no
                                        # collective)
  python bench.py --matrix lj           # products past int32 nnz(C) (the reference's
                                        # `int nnzC`, src/tilespgemm-cuda.h:2327) run as
                                        # sequential tile-row blocks of <= 1.5e9 products
                                        # each; every block's C stays on its device
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

# CPUs this process may run on, read before any OpenMP runtime binds the main
# thread (with OMP_PROC_BIND the main thread's own mask shrinks to one CPU)
try:
    _AFFINITY = len(os.sched_getaffinity(0))
except (AttributeError, OSError):
    _AFFINITY = None
# CPU baseline threads stay on neighbouring cores; must be set
# before any OpenMP runtime (torch's or the oracle's) initialises
os.environ.setdefault("OMP_PROC_BIND", "close")

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "SpGEMM GFLOPS (fp64, C=A^2) + achieved HBM GB/s fraction, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.0  # one xGMI link, per direction (MI355X_MICROARCH.md)
STAGE_STEPS = 3  # untimed steps with the stage events on (bench.py stage_ms)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_matrix(args):
    from spgemm_amd import synth
    if args.mtx:
        from spgemm_amd import tilespgemm as T
        A = T.mmio_allinone(args.mtx)
        T.values_pos_mod10(A)
        m, n, rp, ci, vv = A.csr()
        return m, n, rp, ci, vv, os.path.basename(args.mtx), "real"
    if args.matrix == "mawi":
        m, n, rp, ci, vv = synth.mawi(scale=args.scale)
        tag = "mawi-synthetic" + (f"x{args.scale:g}" if args.scale != 1.0 else "")
        return m, n, rp, ci, vv, tag, "synthetic"
    m, n, rp, ci, vv = synth.GENERATORS[args.matrix]()
    return m, n, rp, ci, vv, args.matrix + "-synthetic", "synthetic"


def transpose_host(m, n, rp, ci, vv):
    import scipy.sparse as sp
    T = sp.csr_matrix((vv, ci, rp), shape=(m, n)).T.tocsr()
    T.sort_indices()
    return n, m, T.indptr.astype(np.int32), T.indices.astype(np.int32), T.data


def nnzcub_rows(rp_a, ci_a, rp_b, r0, r1):
    blen = np.diff(rp_b.astype(np.int64))
    s, e = int(rp_a[r0]), int(rp_a[r1])
    return int(blen[ci_a[s:e]].sum())


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _strided_rows(m, rp, ci, vv, stride):
    """Rows 0, stride, 2*stride, ... of a CSR as a standalone CSR (a row sample
    that keeps the per-row cost distribution of the whole matrix)."""
    rows = np.arange(0, m, max(1, int(stride)), dtype=np.int64)
    rp64 = rp.astype(np.int64)
    lens = rp64[rows + 1] - rp64[rows]
    rps = np.concatenate([[0], np.cumsum(lens)])
    idx = np.repeat(rp64[rows] - rps[:-1], lens) + np.arange(int(rps[-1]), dtype=np.int64)
    return len(rows), rps.astype(np.int32), ci[idx], vv[idx]


def _timed_sample(fn, m, rp, ci, vv, rpb, budget_s):
    """fn(A sample) timed on the whole A when a probe predicts it fits budget_s,
    else on a strided row sample sized to it ("time a strided
    row sample and extrapolate"); (stride, products of the sample, seconds,
    fn's result on the sample)."""
    blen = np.diff(rpb.astype(np.int64))
    probe = max(1, m // 2000)
    sub = _strided_rows(m, rp, ci, vv, probe)
    t0 = time.perf_counter()
    res = fn(*sub)
    t = time.perf_counter() - t0
    stride = probe
    while True:  # (small samples overestimate: fixed per-call costs) -- refine once or twice
        est_full = t * stride
        nxt = 1 if est_full <= budget_s else int(np.ceil(est_full / budget_s))
        if nxt >= stride and stride != probe:
            break
        stride = min(nxt, stride)
        sub = _strided_rows(m, rp, ci, vv, stride) if stride > 1 else (m, rp, ci, vv)
        t0 = time.perf_counter()
        res = fn(*sub)
        t = time.perf_counter() - t0
        if stride == 1:
            break
    return stride, int(blen[sub[2]].sum()), t, res


def _row_chunks(mm, r, c, blen, cap=1.5e9):
    """[r0, r1) row ranges of a CSR whose intermediate products stay <= cap each
    (products bound nnz(C): every chunk's C fits the oracle's int32 row pointers)."""
    cum = np.concatenate([[0], np.cumsum(blen[c])])[r.astype(np.int64)]
    out, r0 = [], 0
    while r0 < mm:
        r1 = int(np.searchsorted(cum, cum[r0] + cap, side="right")) - 1
        r1 = min(mm, max(r1, r0 + 1))
        out.append((r0, r1))
        r0 = r1
    return out


def cpu_baseline(m, n, rp, ci, vv, mb, nb, rpb, cib, vvb, budget_s):
    """The reference's CPU SPA (spgemm_serialref_spa_new.h:7-105, clean-room oracle
    restatement, both passes; symbolic only) on the same workload -- whole when it
    fits the budget, else a strided row sample marked "extrapolated" -- plus the
    oracle's numeric Gustavson timed beside it.  The SPA runs in
    row chunks of <= 1.5e9 products so that every chunk's C fits int32 row
    pointers (the oracle's, as the reference's `int nnzC`); its nnz(C) is
    reported (the whole C's when every row ran)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle as O
    B = O.OMat.from_csr(mb, nb, rpb, cib, vvb)
    blen = np.diff(rpb.astype(np.int64))

    def spa(mm, r, c, v):
        A = O.OMat.from_csr(mm, n, r, c, v)
        nnz = 0
        for r0, r1 in _row_chunks(mm, r, c, blen):
            nnz += len(O.spa(A, B, r0, r1)[1])
        return nnz

    def gus(mm, r, c, v):
        A = O.OMat.from_csr(mm, n, r, c, v)
        return O.gustavson_rows(A, B, 0, mm)

    stride, cub, t, spa_nnz = _timed_sample(spa, m, rp, ci, vv, rpb, budget_s)
    nstride, ncub, nt, _ = _timed_sample(gus, m, rp, ci, vv, rpb, budget_s / 2)
    thr = O.num_threads()
    nproc = os.cpu_count()
    affinity = _AFFINITY
    # threads actually used: the OpenMP team (OMP_NUM_THREADS, which the GPU pool
    # sets to the box's CPU share per GPU), capped by the process's affinity mask
    cores = min(thr, affinity) if affinity else thr

    def what(st):
        return ("all rows" if st == 1 else
                f"extrapolated from a strided sample: every {st}-th row ({100.0 / st:.2g} % of the rows)")
    return {"value": round(2.0 * cub / t / 1e9, 4), "unit": "GFLOPS", "cores": cores, "omp_threads": thr,
            "nproc": nproc, "affinity_cpus": affinity,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "kind": "port", "extrapolated": stride > 1, "seconds": round(t, 3),
            "nnzC": int(spa_nnz), "nnzC_of": "all rows" if stride == 1 else f"the sample (every {stride}-th row)",
            "sample": f"spgemm_spa restatement (count+fill passes, symbolic), {what(stride)} of {m} "
                      f"({cub} intermediate products), {t:.1f} s; {thr} OpenMP threads on {cores} "
                      f"usable CPU(s) of {nproc} (affinity mask {affinity}; OMP_PROC_BIND="
                      f"{os.environ.get('OMP_PROC_BIND', 'unset')}) on {_cpu_model()}",
            "numeric": {"value": round(2.0 * ncub / nt / 1e9, 4), "unit": "GFLOPS", "extrapolated": nstride > 1,
                        "sample": f"oracle Gustavson (dense-row accumulator, fp64 values), {what(nstride)}, "
                                  f"{nt:.1f} s"}}


def tiled_leg(m, n, rp, ci, vv, mb, nb, rpb, cib, vvb, aat, tm, nnzcub, reps=3, warmup=1):
    """The reference-layout drop-in path, timed like the reference: csr2tile of A
    (row-major) and B (col-major) on the host API, then tsg_tilespgemm -- tiles
    in, the reference's tiled C out (tile-pattern step 1 incl. empty C tiles,
    step 2 masks + scan, step 3 values) -- whose time_tile is the reference's
    timed region (steps 1-3 incl. device allocations, src/tilespgemm-cuda.h:
    2358-2747).  Host<->device copies of the tile arrays are outside it, as in
    the reference (its H2D precedes tstart, its D2H follows tend)."""
    from spgemm_amd import tilespgemm as T
    os.environ["TSG_QUIET"] = "1"  # the reference's printf lines would pollute stdout
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    B = T.Matrix.from_csr(mb, nb, rpb, cib, vvb)
    T.csr2tile_row_major(A, tm, tm)
    T.csr2tile_col_major(B, tm, tm)
    runs = []
    for _ in range(reps + max(1, warmup)):
        Cm, info = T.tilespgemm(A, B, tm, tm, nnzCub=nnzcub)
        runs.append((info, Cm.s.numtile))
        del Cm
    runs = runs[max(1, warmup):]  # the first call(s) warm the context's caching allocator
    med = lambda k: float(np.median([r[0][k] for r in runs]))
    t = med("time_tile")
    # the 16x16 CSR route records its step markers only with TSG_STAGE_EVENTS=1
    # (each cost a few us of GPU time): the step times from two untimed calls
    steps = {k: med(k) for k in ("time_step1", "time_step2", "time_step3", "time_malloc")}
    steps_src = "the timed calls"
    if tm == 16 and os.environ.get("TSG_STAGE_EVENTS") != "1":
        os.environ["TSG_STAGE_EVENTS"] = "1"
        try:
            for _ in range(2):
                Cm, info = T.tilespgemm(A, B, tm, tm, nnzCub=nnzcub)
                del Cm
        finally:
            del os.environ["TSG_STAGE_EVENTS"]
        steps = {k: float(info[k]) for k in steps}
        steps_src = "the second of two untimed calls after the timed ones, with TSG_STAGE_EVENTS=1"
    calls = len(runs) + max(1, warmup) + (2 if steps_src != "the timed calls" else 0)  # tsg_tilespgemm calls made
    numblk, nnzc = int(runs[0][1]), int(runs[0][0]["nnzC"])
    # roofline of the timed region (steps 1-3): the reference's byte model
    # (B_alg) and, for context, the bytes of the reference LAYOUT the
    # region must write -- C's tile structure (column + row index), tile_nnz, the
    # per-tile row pointers and masks (tm u16 each, tm/16 mask words per row),
    # the u16 local columns and fp64 values -- plus the A/B tile payloads it reads
    b_alg = 4.0 * (m + 1) + 12.0 * len(ci) + 4.0 * (mb + 1) + 12.0 * len(cib) + 4.0 * (m + 1) + 12.0 * nnzc
    wpr = max(1, tm // 16)
    layout = (4.0 * (m // tm + 2) + 12.0 * numblk + 2.0 * tm * numblk * (1 + wpr) + 10.0 * nnzc
              + 10.0 * (len(ci) + len(cib)))
    return {"t_kern_tiled_ms": round(t, 4), "gflops": round(2.0 * nnzcub / (t * 1e-3) / 1e9, 3),
            "t_step1_ms": round(steps["time_step1"], 4), "t_step2_ms": round(steps["time_step2"], 4),
            "t_step3_ms": round(steps["time_step3"], 4), "t_malloc_ms": round(steps["time_malloc"], 4),
            "step_times_source": steps_src,
            "numblkC": numblk, "nnzC": nnzc, "reps": reps, "tile": tm, "calls_made": calls,
            "step_times_overlap": tm == 16,
            "step_times_note": ("16x16 CSR route: step 1 runs on its own stream beside steps 2-3, so the three "
                                "step times overlap and do not add up to t_kern_tiled_ms (t_malloc_ms, the "
                                "remainder, clamps at 0); the reference's steps run one after another")
                               if tm == 16 else "steps 1-3 in turn",
            "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                         "algorithmic_bytes": int(b_alg), "achieved": round(b_alg / (t * 1e-3) / 1e9, 2),
                         "frac": round(b_alg / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                         "layout_bytes": int(layout), "layout_achieved": round(layout / (t * 1e-3) / 1e9, 2),
                         "layout_frac": round(layout / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                         "note": "B_alg / the timed region (steps 1-3); layout_bytes = the reference tiled C "
                                 "arrays written + the A/B tile payloads read"},
            "path": "tsg_tilespgemm (reference tiled layout in/out; the ./test CLI path)"}


def profile_order(path):
    """Sort key of a profiles/r<round><tag>_* file: the round, then the tag in
    the order tags are handed out (a .. z, then aa .. zz: shorter first)."""
    import re
    mt = re.match(r"r(\d+)([A-Za-z]+)_", os.path.basename(path))
    return (int(mt.group(1)), len(mt.group(2)), mt.group(2)) if mt else (-1, 0, os.path.basename(path))


def pmc_file(workload, explicit=None, root=None):
    """The PMC summary the line's traffic comes from: `explicit` (--pmc-from: the
    profile run of the same build writes it right before its timed run), else the
    newest committed profiles/<round>_pmc.json of the same workload."""
    import glob
    if explicit:
        return explicit if os.path.exists(explicit) else None

    def workload_of(f):
        try:
            return json.load(open(f)).get("_workload")
        except (OSError, ValueError, AttributeError):  # unreadable / partial summary
            return None
    files = sorted(glob.glob(os.path.join(root or REPO, "profiles", "r*_pmc.json")), key=profile_order)
    files = [f for f in files if workload_of(f) == workload]
    return files[-1] if files else None


def pmc_traffic(kernels, path):
    """HBM bytes per call of the `kernels` (name substrings; their per-dispatch
    bytes summed) and of every kernel of the call, from a PMC summary
    (tools/pmc_summary.py: 2*FETCH_SIZE + WRITE_SIZE, separate --pmc passes).
    (unit bytes, all-kernel bytes per call), None where absent."""
    if not path:
        return None, None
    d = json.load(open(path))
    calls = (d.get("_per_call") or {}).get("calls")
    tot, found = 0, False
    for kernel in kernels:  # (the kernels of the unit that ran for this workload)
        hits = [v for k, v in d.items() if kernel in k and isinstance(v, dict) and v.get("hbm_bytes_per_dispatch")]
        found |= bool(hits)
        for v in hits:
            # per call: a kernel dispatched several times per call (sequential row
            # blocks: once per block) counts every dispatch
            per_call = v["dispatches"] / calls if calls and v.get("dispatches") else 1.0
            tot += int(v["hbm_bytes_per_dispatch"]) * max(1.0, per_call)
    allk = (d.get("_per_call") or {}).get("hbm_bytes")
    return (int(tot) if found else None), allk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--matrix", default="webbase", choices=["webbase", "cant", "mc2depi", "lj", "mawi"])
    ap.add_argument("--scale", type=float, default=1.0, help="size factor for the mawi stand-in")
    ap.add_argument("--mtx", default=os.environ.get("TSG_MTX"))
    ap.add_argument("--aat", type=int, default=None)
    ap.add_argument("--tile", type=int, default=16)
    ap.add_argument("--rows", type=int, default=None,
                    help="A = its first ROWS rows (B whole); default: all rows, or for configs whose "
                         "full product exceeds int32 nnz(C) (lj) the largest prefix with nnzCub <= 1.5e9")
    ap.add_argument("--row-start", type=int, default=0,
                    help="with --rows R: A = rows [ROW_START, ROW_START + R) (e.g. the LiveJournal "
                         "stand-in's heaviest row block; B whole)")
    ap.add_argument("--cpu-budget-s", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", action="store_true",
                    help="add a checksum of the (gathered) C of the last step to the JSON line")
    ap.add_argument("--dump", default=None,
                    help="rank 0 saves the (gathered) C of the last step as an .npz (rowptr, col, val), "
                         "outside the timed region (array-level parity tests)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N>1 (nccl = RCCL over xGMI; gloo = host-staged "
                         "rehearsal of the multi-rank path, e.g. several ranks on one GPU)")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="N>1: strong (default, north_star's exchange step) = the fixed product, A's rows "
                         "partitioned by work, B replicated, the RCCL gather of C to rank 0 inside the timed "
                         "region (gather-bound, DESIGN section 5); weak = NOT the north-star metric: every "
                         "rank owns one A-sized row block of the stacked product [A; ...; A]*B (fixed work "
                         "per GPU, C stays distributed, no data-path collective)")
    ap.add_argument("--gather-sub", type=int, default=0,
                    help="N>1 strong: the rows are cut into N x this many pieces of equal products, rank r "
                         "computing piece (s, r) in round s; each round goes to rank 0 straight into the final "
                         "C while the next one computes (dist.RoundGather); 0 = auto: 4 when a rank holds "
                         ">= 2e8 products, else 1")
    ap.add_argument("--block-products", type=float, default=1.5e9,
                    help="row-block size (intermediate products) when the product exceeds int32 "
                         "nnz(C): such products run as sequential row blocks, C kept per block")
    ap.add_argument("--pmc-from", default=None,
                    help="PMC summary (tools/pmc_summary.py) the roofline's traffic comes from; default: the newest "
                         "committed profiles/r*_pmc.json of the same workload")
    ap.add_argument("--leg", default="device", choices=["device", "tiled"],
                    help="tiled: time only the reference-layout drop-in path tsg_tilespgemm (the ./test timed "
                         "region; e.g. under rocprofv3 for its kernel stats) and print its line")
    ap.add_argument("--tiled", type=int, default=None,
                    help="also time the reference-layout host path tsg_tilespgemm (csr2tile tiles "
                         "in, tiled C out; the reference's timed region) -> t_kern_tiled_ms; "
                         "default on at N=1 for matrices with <= 4e8 intermediate products")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dev_id = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_id)
    dist = None
    host_coll = args.backend == "gloo"  # gloo collectives take host tensors
    red_dev = "cpu" if host_coll else "cuda"
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if host_coll:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_id))

    from spgemm_amd.device import Context, DeviceCSR
    from spgemm_amd import dist as tdist

    m, n, rp, ci, vv, name, data_kind = load_matrix(args)
    aat = args.aat if args.aat is not None else (1 if args.matrix == "mc2depi" and not args.mtx else 0)
    if aat:
        mb, nb, rpb, cib, vvb = transpose_host(m, n, rp, ci, vv)
    else:
        mb, nb, rpb, cib, vvb = m, n, rp, ci, vv
    tm = args.tile
    full_m = m
    if args.leg == "tiled":
        # the drop-in path alone: csr2tile on the host API (untimed, as in the reference),
        # then tsg_tilespgemm's timed region (steps 1-3 with allocations) per call
        if args.rows is not None:
            m, rp, ci, vv = args.rows, rp[:args.rows + 1].copy(), ci[:rp[args.rows]].copy(), vv[:rp[args.rows]].copy()
        cub = nnzcub_rows(rp, ci, rpb, 0, m)
        tl = tiled_leg(m, n, rp, ci, vv, mb, nb, rpb, cib, vvb, aat, tm, cub, reps=args.steps, warmup=args.warmup)
        out = {"metric": METRIC, "value": tl["gflops"], "unit": "GFLOPS", "n_gpus": 1, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": tl["t_kern_tiled_ms"], "higher_is_better": True,
               "scaling": "single", "vs_baseline": None, "dtype": "f64", "data": data_kind,
               "config": {"workload": f"{name} C=A{'*A^T' if aat else '^2'} fp64, tsg_tilespgemm {tm}x{tm} "
                                      f"(tiles in -> tiled C out; the reference's timed region)",
                          "m": m, "nnzA": int(len(ci)), "nnzCub": cub, "nnzC": tl["nnzC"], "path": "tiled"},
               "roofline": tl["roofline"], "tiled": tl, "calls_made": tl["calls_made"]}
        # HBM traffic of the call from a PMC summary of the same command (tools/profile.sh
        # --leg tiled): every kernel's bytes over the calls, which also spreads the
        # one-time csr2tile of A and B (outside the timed region) over the calls
        pfile = pmc_file(out["config"]["workload"], args.pmc_from)
        rl = out["roofline"]
        rl["traffic_all_kernels"] = None
        if pfile:
            # the compute kernels' bytes per call; the runtime's copy kernels
            # (__amd_rocclr_*: the tiles' uploads and the tiled C's downloads,
            # outside the timed region as in the reference) left out
            d = json.load(open(pfile))
            calls = (d.get("_per_call") or {}).get("calls")
            tot = sum(v["hbm_bytes_per_dispatch"] * v["dispatches"] for k, v in d.items()
                      if isinstance(v, dict) and v.get("hbm_bytes_per_dispatch") and v.get("dispatches")
                      and not k.startswith("__amd_rocclr"))
            rl["traffic_all_kernels"] = round(tot / calls) if calls else None
        allk = rl["traffic_all_kernels"]
        rl["traffic_over_b_alg"] = round(allk / rl["algorithmic_bytes"], 3) if allk else None
        rl["layout_traffic_ratio"] = round(allk / rl["layout_bytes"], 3) if allk else None
        rl["traffic_source"] = os.path.relpath(pfile, REPO) if pfile else None
        print(json.dumps(out), flush=True)
        return
    blen_b = np.diff(rpb.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen_b[ci])])[rp]  # nnzCub of row prefixes
    rows = args.rows
    if rows is None and args.matrix == "mawi" and not args.mtx and cum[-1] > 1e12:
        # mawi's hub makes the full A^2 ~1e14 products (~2000 s a step): the largest
        # row prefix within one int32 C, as SURVEY §8d prescribes for infeasible sizes
        rows = int(np.searchsorted(cum, args.block_products, side="right") - 1) // tm * tm
        log(f"full product infeasible (nnzCub {int(cum[-1])}); using rows [0,{rows})")
    if rows is not None and args.row_start > 0:
        r0 = min(args.row_start, m)
        r1 = min(m, r0 + rows)
        rows_, rp_, ci_, vv_ = tdist.slice_rows(m, rp, ci, vv, r0, r1)
        m, rp, ci, vv = rows_, rp_, ci_.copy(), vv_.copy()
        cum = cum[r0:r1 + 1] - cum[r0]
        name = f"{name} rows[{r0},{r1}) of {full_m}"
    elif rows is not None and rows < m:
        m, rp, ci, vv = rows, rp[:rows + 1].copy(), ci[:rp[rows]].copy(), vv[:rp[rows]].copy()
        cum = cum[:rows + 1]
        name = f"{name} rows[0,{rows}) of {full_m}"
    nnzcub_full = int(cum[-1])
    weak = world > 1 and args.scaling == "weak"
    nnzcub_total = nnzcub_full * world if weak else nnzcub_full
    # products past int32 nnz(C) (the reference's `int nnzC`): sequential row
    # blocks of <= block_products each, every block's C kept on the device
    blocked = nnzcub_full > args.block_products
    gather = world > 1 and not weak and not blocked
    nsub = 1
    if gather:
        # the overlapped gather: rows cut into world x nsub pieces of ~equal products
        # (row granularity), rank r computing piece (s, r) in round s (dist.RoundGather)
        nsub = args.gather_sub or (4 if nnzcub_full / world >= 2e8 else 1)
    if world > 1 and not weak:
        pieces = tdist.row_pieces(cum, m, world, nsub)
        my_pieces = [pieces[s][rank] for s in range(nsub)]
    else:
        pieces, my_pieces = None, [(0, m)]
    r_lo, r_hi = my_pieces[0][0], my_pieces[-1][1]  # (blocked / single: one contiguous range)
    blocks = tdist.product_blocks(cum, r_lo, r_hi, args.block_products, tm) if blocked else my_pieces
    dA_blocks = []
    for (b0, b1) in blocks:
        mb_, rpb_, cib_, vvb_ = tdist.slice_rows(m, rp, ci, vv, b0, b1)
        dA_blocks.append((b0, b1, DeviceCSR.from_host(mb_, n, rpb_, cib_, vvb_)))
    if len(dA_blocks) == 1 and not aat and dA_blocks[0][1] - dA_blocks[0][0] == full_m and m == full_m:
        dB = dA_blocks[0][2]
    else:
        dB = DeviceCSR.from_host(mb, nb, rpb, cib, vvb)
    ctx = Context(dev_id)
    torch.cuda.synchronize()
    if blocked:
        log(f"rank {rank}: {len(blocks)} row block(s) of <= {args.block_products:.3g} products, C kept per block")

    gathered = [None]
    gather_ms = []
    compute_ms = []  # per step: this rank's pieces computed (before the gather's exposed wait)
    calls_made = [0]  # device passes this process makes (one_step calls), for the PMC per-call accounting
    sg = None
    if gather:
        # one gatherer for every step: rank 0's C arrays are sized from the gathered
        # nnz counts in the warmup and reused; the counts travel on a host (gloo) group
        meta = dist.new_group(backend="gloo")
        sg = tdist.RoundGather(rank, world, pieces, 0, device="cpu" if host_coll else "cuda", meta_group=meta)

    # B's rows checked once (outside the timed steps; every step's first block
    # checks again inside its own call): the later row blocks of a step skip it
    b_ok = len(dA_blocks) > 1 and ctx.rows_sorted(dB)

    def one_step():
        sts, nnz = [], 0
        c = None
        calls_made[0] += 1
        s0 = time.perf_counter()
        if gather:
            # the rounds in turn, each piece handed to the gather as soon as its C is
            # complete (the context keeps every piece's C until the step ends)
            ctx.reset()
            gathered[0] = None
            sg.reset()
            for s, (_, _, dAb) in enumerate(dA_blocks):
                c, st = ctx.spgemm(dAb, dB, tm, tm, b_sorted=s > 0 and b_ok, raw=True)
                sts.append(st)
                nnz += c.nnz
                cv = ctx.view_torch(c)  # zero-copy views of the context-owned C
                if host_coll:
                    sg.push(s, cv.rowptr.cpu(), cv.col.cpu(), cv.val.cpu(), nnz=c.nnz)
                else:
                    sg.push(s, cv.rowptr, cv.col, cv.val, nnz=c.nnz)
            g0 = time.perf_counter()
            compute_ms.append((g0 - s0) * 1e3)  # (ctx.spgemm returns with C complete: host time = compute)
            gathered[0] = sg.finish()
            if not host_coll:
                torch.cuda.synchronize()
            gather_ms.append((time.perf_counter() - g0) * 1e3)  # (the last round's, not hidden behind compute)
        else:
            for bi, (_, _, dAb) in enumerate(dA_blocks):
                ctx.reset()
                # (row blocks over one B: B's sortedness checked once per step, by the
                # first block's call; the others skip it -- tsg_dev_spgemm_sorted_b)
                c, st = ctx.spgemm(dAb, dB, tm, tm, b_sorted=bi > 0 and b_ok, raw=True)  # returns with C complete
                sts.append(st)
                nnz += c.nnz
            compute_ms.append((time.perf_counter() - s0) * 1e3)
        # (the blocks' raw tsg_stats: merged by merge_stats after the timed steps,
        # not inside them -- at mc2depi's 0.2 ms a step, the dict work was ~5 %)
        return c, sts, nnz

    def merge_stats(sts):
        sts = [s.as_dict() for s in sts]
        st = {k: sum(s[k] for s in sts) for k in sts[0]}
        # (labels, not sums: the path every block took, -1 for "no C tiles")
        paths = {int(s["path"]) for s in sts}
        st["path"] = paths.pop() if len(paths) == 1 else -1
        for k in ("numtileA", "numblkC"):
            if k in st and all(s[k] == -1 for s in sts):
                st[k] = -1
        return st

    for _ in range(args.warmup):
        one_step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    stats = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        c, st, nnz_rank = one_step()
        stats.append(st)
    torch.cuda.synchronize()
    stats = [merge_stats(x) for x in stats]  # (after the clock; see merge_stats)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    compute_timed = compute_ms[-args.steps:]  # (the timed steps' compute times)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        nz = torch.tensor([nnz_rank], dtype=torch.int64, device=red_dev)
        dist.all_reduce(nz)
        nnzC = int(nz.item())
    else:
        nnzC = nnz_rank
    work_share = None
    my_products = float(sum(cum[b] - cum[a] for a, b in my_pieces))
    if dist:
        # each rank's share of the intermediate products (its rows' work) and the
        # max/mean imbalance of the partition
        w = torch.tensor([my_products], dtype=torch.float64, device=red_dev)
        allw = [torch.zeros_like(w) for _ in range(world)]
        dist.all_gather(allw, w)
        ws = [float(x.item()) for x in allw]
        mean = sum(ws) / world
        work_share = {"products": [int(x) for x in ws],
                      "max_over_mean": round(max(ws) / mean, 4) if mean > 0 else None}
        if not weak and mean > 0:
            # the heaviest single row against a rank's fair share (the partition cuts
            # between rows: a row heavier than the share would bound the imbalance)
            prow = np.diff(cum)
            work_share["max_row_over_mean"] = round(float(prow.max()) / mean, 6) if len(prow) else 0.0
    ms_per_step = elapsed * 1e3 / args.steps
    gflops = 2.0 * nnzcub_total * args.steps / elapsed / 1e9
    scale_model = None
    if dist:
        # what bounds this N: every rank's compute time per step, the bytes each
        # peer sends to rank 0 over its own xGMI link and, for the
        # gather, the single-GPU time of the same product measured on rank 0
        # (outside the timed region) -> the ceiling t_1 / max(compute_N, floor)
        rows_mine = sum(b - a for a, b in my_pieces)
        mine = torch.tensor([float(rows_mine), float(nnz_rank), float(np.median(compute_timed))],
                            dtype=torch.float64, device=red_dev)
        allm = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allm, mine)
        rows_r = [int(x[0].item()) for x in allm]
        nnz_r = [int(x[1].item()) for x in allm]
        comp_r = [round(float(x[2].item()), 4) for x in allm]
        t1_ms = None
        if gather and rank == 0:
            dA_full = DeviceCSR.from_host(m, n, rp, ci, vv)
            ts = []
            for _ in range(3):
                ctx.reset()
                q0 = time.perf_counter()
                ctx.spgemm(dA_full, dB, tm, tm)  # (returns with C complete)
                ts.append((time.perf_counter() - q0) * 1e3)
            ctx.reset()
            del dA_full
            t1_ms = float(np.median(ts[1:]))  # (the first call grows the context's pool)
        dist.barrier()
        peer_bytes = [4.0 * (rows_r[r] + nsub) + 12.0 * nnz_r[r] for r in range(1, world)] if gather else []
        floor_ms = max(peer_bytes) / (XGMI_LINK_GBS * 1e9) * 1e3 if peer_bytes else None
        bound = max([max(comp_r)] + ([floor_ms] if floor_ms else []))
        scale_model = {
            "compute_ms": comp_r,
            "compute_note": ("per rank, median over the timed steps: its pieces' device passes (host time to the "
                             "last piece's C complete; ctx.spgemm is synchronous), without the exposed gather"),
            "rows": rows_r, "nnzC": nnz_r,
            "rank0_received_bytes": int(sum(peer_bytes)) if gather else None,
            "max_peer_bytes": int(max(peer_bytes)) if peer_bytes else None,
            "link_GBps": XGMI_LINK_GBS,
            "gather_floor_ms": round(floor_ms, 4) if floor_ms is not None else None,
            "gather_floor_note": ("the largest peer's C rows (4 B per row pointer + 12 B per nonzero) over one "
                                  "xGMI link into rank 0; the peers send in parallel, each on its own link")
                                 if gather else "no gather: C stays distributed",
            "t1_ms": round(t1_ms, 4) if t1_ms is not None else None,
            "t1_source": ("rank 0: the whole product on its own GPU after the timed steps (median of 2 "
                          "calls after one warm call)") if t1_ms is not None else None,
            "ceiling_speedup": round(t1_ms / bound, 3) if t1_ms and bound > 0 else None,
            "ceiling_note": "t1_ms / max(max(compute_ms), gather_floor_ms): perfect overlap of the rounds",
            "measured_speedup": round(t1_ms / ms_per_step, 3) if t1_ms else None,
        }

    med = {k: float(np.median([s[k] for s in stats])) for k in stats[0]}
    mins = {k: float(np.min([s[k] for s in stats])) for k in ("t_e2e_ms", "t_kern_ms")}
    # the stage breakdown from untimed steps with the stage events on
    # (TSG_STAGE_EVENTS=1): the timed steps record only the kernel bracket (its
    # time is the roofline's kernel_ms) -- each stage marker on the stream cost
    # ~2-3 us of GPU time, which the timed steps do not pay.  The median over
    # STAGE_STEPS such steps (the first of them is not dropped: warm by then).
    stage_src = "timed steps (TSG_STAGE_EVENTS=1 set by the caller)"
    if os.environ.get("TSG_STAGE_EVENTS") != "1":
        n_gm = len(gather_ms)
        os.environ["TSG_STAGE_EVENTS"] = "1"
        st_stages = []
        try:
            for _ in range(STAGE_STEPS):
                st_stages.append(merge_stats(one_step()[1]))
        finally:
            del os.environ["TSG_STAGE_EVENTS"]
        del gather_ms[n_gm:]
        for k in ("t_csr2tile_ms", "t_step1_ms", "t_step2_ms", "t_step3_ms", "t_tile2csr_ms", "t_kern_ms",
                  "t_malloc_ms"):
            med[k] = float(np.median([x[k] for x in st_stages]))
        mins["t_kern_ms"] = float(np.min([x["t_kern_ms"] for x in st_stages]))
        stage_src = (f"median of {STAGE_STEPS} untimed steps after the timed ones, with TSG_STAGE_EVENTS=1 "
                     "(t_kern_ms and gflops_kern included)")
    dev_ms = med["t_csr2tile_ms"] + med["t_step1_ms"] + med["t_step2_ms"] + med["t_step3_ms"] + med["t_tile2csr_ms"]
    # SURVEY §8d algorithmic bytes (src/external/cusparse/main.cu:205-208), this rank's share
    mrank = sum(b - a for a, b in my_pieces)
    nnza_rank = int(sum(int(rp[b]) - int(rp[a]) for a, b in my_pieces))
    nb_calls = 1 if gather else len(blocks)  # (the gather's sub-blocks: B counted once, as one call)
    b_survey = (4.0 * (mrank + nb_calls) + 12.0 * nnza_rank + (4.0 * (mb + 1) + 12.0 * len(cib)) * nb_calls
                + 4.0 * (mrank + nb_calls) + 12.0 * nnz_rank)
    # the same with B's term the rows A references (each once per call) instead of
    # all of B: a row block (mawi's prefix, a LiveJournal block) reads only those,
    # and once a kernel reads a shared run once (the dominant-run fill) B_survey's
    # whole-B term would put "achieved" past the HBM peak; equal to B_survey for a
    # full product whose A references every B row
    blen_b = np.diff(rpb.astype(np.int64))
    b_ref = 0.0
    for call in ([my_pieces] if gather else [[bk] for bk in blocks]):
        used = np.zeros(mb, dtype=bool)
        for a, b in call:
            used[ci[int(rp[a]):int(rp[b])]] = True
        b_ref += 12.0 * float(blen_b[used].sum()) + 8.0 * float(used.sum())
    b_alg = 4.0 * (mrank + nb_calls) + 12.0 * nnza_rank + b_ref + 4.0 * (mrank + nb_calls) + 12.0 * nnz_rank
    achieved_pipe = b_alg / (dev_ms * 1e-3) / 1e9 if dev_ms > 0 else 0.0  # (0: stage events off)
    # context only (never the graded figure): + one fp64 value and one u16 local column
    # per intermediate product of this rank (SURVEY §8d B_stream)
    b_stream = b_alg + 10.0 * my_products
    # dominant kernel (reads the CSR operands, builds the C rows = B_alg's terms),
    # timed with HIP events on the call's stream: the staged pipeline's step-3
    # numeric kernel, or the row-merge path's numeric phase (its class kernels
    # S, M1-M4, H on 4 streams, forked from and joined to the call's stream)
    k3_ms = med["t_step3_kernel_ms"]
    achieved = b_alg / (k3_ms * 1e-3) / 1e9
    path_id = int(med["path"])
    path_name = {-1: "mixed", 0: "tiles", 2: "band", 3: "rows"}.get(path_id, str(path_id))
    workload = f"{name} C=A{'*A^T' if aat else '^2'} fp64 (device CSR in -> device CSR out), path {path_name}"
    if path_id == 3:
        kernel_desc = ("row-merge numeric phase (class H: k_rows_bitmap / hub rows k_rows_w*, k_rows_dr_*; "
                       "k_rows_merge x5 classes, k_rows_small x2; in turn; with windowed or dominant-run rows "
                       "to the end of their fills into C after the row scan): B_alg (A + the B rows A references + C) / HIP-event "
                       "phase time")
        unit_kernels = ["k_rows_small", "k_rows_merge", "k_rows_bitmap", "k_rows_wplan", "k_rows_wcount",
                        "k_rows_wscatter", "k_rows_wunit", "k_rows_wgather", "k_rows_dr_", "k_rows_ob"]
    elif path_id == 2:
        kernel_desc = ("band row kernel k_band_rows (one workgroup per C row, LDS window accumulator): "
                       "B_alg (A + the B rows A references + C) / HIP-event kernel time")
        unit_kernels = ["k_band_rows"]
    else:
        kernel_desc = "step-3 numeric kernel (fused tile2csr): B_alg (A + the B rows A references + C) / HIP-event kernel time"
        unit_kernels = ["k_step3"]
    pfile = pmc_file(workload, args.pmc_from)
    traffic, traffic_all = pmc_traffic(unit_kernels, pfile)
    traffic_src = os.path.relpath(pfile, REPO) if pfile else None
    chk = None
    if args.check and not gather:
        # checksum of this rank's C (every block), recomputed outside the timed region;
        # row pointers summed as the one global CSR would hold them
        acc = np.zeros(4)
        off = 0
        calls_made[0] += 1
        for (_, _, dAb) in dA_blocks:
            ctx.reset()
            cb, _ = ctx.spgemm(dAb, dB, tm, tm)
            g_rp, g_ci, g_vv = ctx.to_host(cb)[2:]
            acc += [float(len(g_ci)), float(g_rp[:-1].astype(np.int64).sum() + off * (len(g_rp) - 1)),
                    float(g_ci.astype(np.int64).sum()), float(g_vv.sum())]
            off += len(g_ci)
        rows_rank = mrank
        if weak:  # every rank's block of the stacked product is the same C
            chk = acc.copy()
            chk[1] += off
            t = torch.tensor(chk, dtype=torch.float64, device=red_dev)
            lo, hi = t.clone(), t.clone()
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            assert torch.equal(lo, hi), "weak scaling: rank C blocks differ"
        elif world > 1:  # blocked strong: C stays distributed; shift by the ranks before
            cnt = torch.tensor([float(off), float(rows_rank)], dtype=torch.float64, device=red_dev)
            allc = [torch.zeros_like(cnt) for _ in range(world)]
            dist.all_gather(allc, cnt)
            before = sum(float(allc[q][0]) for q in range(rank))
            acc[1] += before * rows_rank
            t = torch.tensor(acc, dtype=torch.float64, device=red_dev)
            dist.all_reduce(t)
            chk = t.cpu().numpy()
            chk[1] += sum(float(c[0]) for c in allc)  # rowptr[m] = nnz(C)
        else:
            chk = acc
            chk[1] += off
    if args.dump and world == 1 and not blocked:
        calls_made[0] += 1
        ctx.reset()
        cb, _ = ctx.spgemm(dA_blocks[0][2], dB, tm, tm)
        g_rp, g_ci, g_vv = ctx.to_host(cb)[2:]
        np.savez(args.dump, rowptr=g_rp, col=g_ci, val=g_vv)
    elif args.dump and gather and rank == 0:
        g_rp, g_ci, g_vv = (x.cpu().numpy() for x in gathered[0])
        np.savez(args.dump, rowptr=g_rp, col=g_ci, val=g_vv)
    tiled = None
    want_tiled = args.tiled if args.tiled is not None else (world == 1 and nnzcub_full <= 4e8)
    if want_tiled and rank == 0 and world == 1:
        tiled = tiled_leg(m, n, rp, ci, vv, mb, nb, rpb, cib, vvb, aat, tm, nnzcub_full)
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(m, n, rp, ci, vv, mb, nb, rpb, cib, vvb, args.cpu_budget_s)
            except Exception as e:  # the baseline is reported, never required
                log(f"cpu baseline failed: {e!r}")
        if world == 1:
            par = "single" + (f" ({len(blocks)} sequential row blocks, C per block)" if blocked else "")
        elif weak:
            par = f"stacked-row-block{world} (B replicated, C distributed)"
        elif gather:
            par = f"row-pieces{world}x{nsub} + RCCL gather"
        else:
            par = f"row-block{world} x {len(blocks)} sequential blocks (C distributed: past one int32 CSR)"
        out = {
            "metric": METRIC, "value": round(gflops, 3), "unit": "GFLOPS", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "single" if world == 1 else args.scaling,
            "vs_baseline": None, "dtype": "f64", "data": data_kind,
            "config": {"workload": workload,
                       "m": m * world if weak else m, "m_per_rank": m if weak else None,
                       "nnzA": int(len(ci)) * (world if weak else 1), "nnzCub": nnzcub_total, "nnzC": nnzC,
                       "path": path_name,
                       "numtileA": int(med["numtileA"]),
                       "numblkC": int(med["numblkC"]),
                       "numblkC_kind": ("element-level C tiles (non-empty 16x16 tiles of C; the reference's "
                                        "tile-pattern step 1 also lists empty ones, see t_kern_tiled)") if path_id == 0
                                       else "-1: this path builds no C tiles (the reference-layout tiled C: see tiled)",
                       "row_blocks": 1 if gather else len(blocks),
                       "gather_rounds": nsub if gather else None,
                       "parallelism": par},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": kernel_desc,
                         "algorithmic_bytes": int(b_alg), "kernel_ms": round(k3_ms, 4),
                         "algorithmic_bytes_def": ("A + the B rows A references (once per call) + C, "
                                                   "12 B per nonzero + row pointers; B_survey (all of B) beside"),
                         "algorithmic_bytes_survey": int(b_survey),
                         "pipeline": {"achieved": round(achieved_pipe, 2),
                                      "frac": round(achieved_pipe / HBM_PEAK_GBS, 5),
                                      "device_ms": round(dev_ms, 4)},
                         # the whole pass as the driver times it: B_alg / ms_per_step (this rank's
                         # bytes over the max-over-ranks step time), and every kernel's measured
                         # HBM bytes of one call against B_alg
                         "pass": {"achieved": round(b_alg / (ms_per_step * 1e-3) / 1e9, 2),
                                  "frac": round(b_alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                                  "ms": round(ms_per_step, 4),
                                  "traffic_all_kernels": traffic_all,
                                  "traffic_all_over_b_alg": round(traffic_all / b_alg, 3) if traffic_all else None},
                         "traffic_over_b_alg": round(traffic / b_alg, 3) if traffic else None,
                         "stream_bytes": int(b_stream),
                         "stream_achieved": round(b_stream / (k3_ms * 1e-3) / 1e9, 2)},
            "stage_ms": {k: round(med[k], 4) for k in ("t_csr2tile_ms", "t_step1_ms", "t_step2_ms",
                                                        "t_step3_ms", "t_step3_kernel_ms", "t_tile2csr_ms", "t_malloc_ms",
                                                        "t_kern_ms", "t_e2e_ms")},
            "stage_ms_min": {k: round(v, 4) for k, v in mins.items()},
            "stage_ms_source": stage_src,
            "gather_ms": round(float(np.median(gather_ms[-args.steps:])), 4) if gather_ms else None,
            "gather_note": ("rank 0: the gather's exposed part (after the last sub-block's compute; the "
                            "earlier sub-blocks travel while the next ones compute)") if gather_ms else None,
            "work_share": work_share,
            "scale_model": scale_model,
            "calls_made": calls_made[0],
            "gflops_kern": (round(2.0 * nnzcub_total / (med["t_kern_ms"] * 1e-3) / 1e9, 3)
                            if world == 1 and med["t_kern_ms"] > 0 else None),
            "tiled": tiled,
            "cpu_baseline": cpu,
        }
        if args.check:
            if chk is not None:
                out["check"] = {"nnz": int(chk[0]), "rowptr_sum": int(chk[1]), "col_sum": int(chk[2]),
                                "val_sum": float(chk[3])}
            else:
                g_rp, g_ci, g_vv = (x.cpu().numpy() for x in gathered[0])
                out["check"] = {"nnz": int(len(g_ci)), "rowptr_sum": int(g_rp.astype(np.int64).sum()),
                                "col_sum": int(g_ci.astype(np.int64).sum()), "val_sum": float(g_vv.sum())}
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
