"""Multi-GPU TileSpGEMM: one process per GPU.

C's tile row i depends only on A's tile row i and all of B, so A is split into
contiguous blocks of tile rows of equal WORK (prefix sum of the per-tile-row
intermediate products, the quantity nsparse's set_intprod_num bins on,
src/spgemm_nsparse_kernel.h:135-151), B is replicated, every rank runs the full
device pipeline on its block, and the single exchange step is a gather of the
C row blocks to rank 0 (point-to-point sends over RCCL/xGMI; each peer uses its
own link into the root, RCCL has no gatherv).  Backend-agnostic: the same code
runs on gloo (CPU tensors, tests) and nccl (= RCCL on ROCm, GPU tensors).
"""
import numpy as np


def tile_row_work(rowptr_a, col_a, rowptr_b, m, tile_m):
    """Element-level intermediate products per A tile row (sum of B row lengths)."""
    blen = np.diff(rowptr_b.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen[col_a])])
    rp = np.asarray(rowptr_a, dtype=np.int64)
    per_row = cum[rp[1:]] - cum[rp[:-1]]
    tilem = (m + tile_m - 1) // tile_m
    pad = np.zeros(tilem * tile_m, dtype=np.int64)
    pad[:m] = per_row
    return pad.reshape(tilem, tile_m).sum(axis=1)


def partition_tile_rows(work, world):
    """Contiguous [begin, end) tile-row ranges of ~equal work (+1 per row so
    empty rows still spread)."""
    w = np.asarray(work, dtype=np.float64) + 1.0
    cum = np.concatenate([[0.0], np.cumsum(w)])
    bounds = [0]
    for r in range(1, world):
        bounds.append(int(np.searchsorted(cum, cum[-1] * r / world, side="left")))
    bounds.append(len(w))
    bounds = np.maximum.accumulate(np.array(bounds))
    return [(int(bounds[r]), int(bounds[r + 1])) for r in range(world)]


def product_blocks(cum, r_lo, r_hi, cap, tile_m):
    """Split rows [r_lo, r_hi) into consecutive tile-row-aligned blocks of at
    most `cap` intermediate products each (cum = nnzCub of the row prefixes,
    length m+1).  Products past the reference's int32 nnz(C)
    (src/tilespgemm-cuda.h:2327) run as such blocks, one after another; a single
    tile row heavier than `cap` becomes a block of its own."""
    cum = np.asarray(cum, dtype=np.int64)
    m = len(cum) - 1
    bounds = [r_lo]
    while bounds[-1] < r_hi:
        lo = bounds[-1]
        nxt = int(np.searchsorted(cum, cum[lo] + cap, side="right") - 1) // tile_m * tile_m
        bounds.append(min(r_hi, m, max(nxt, lo + tile_m)))
    if len(bounds) == 1:
        bounds.append(r_hi)
    return list(zip(bounds[:-1], bounds[1:]))


def slice_rows(m, rowptr, col, val, r0, r1):
    """Rows [r0, r1) of a CSR as a standalone CSR (row pointers rebased)."""
    r0, r1 = max(0, min(r0, m)), max(0, min(r1, m))
    s, e = int(rowptr[r0]), int(rowptr[r1])
    rp = (rowptr[r0:r1 + 1] - s).astype(np.int32)
    return r1 - r0, rp, col[s:e], val[s:e]


def gather_csr_blocks(rowptr, col, val, rank, world, device=None):
    """Gather CSR row blocks (torch tensors on `device`) to rank 0.

    Returns (rowptr, col, val) of the concatenated matrix on rank 0, None elsewhere.
    One all_gather of the per-rank (rows, nnz) counts, then point-to-point
    sends of each block's arrays into the root's slices."""
    import torch
    import torch.distributed as dist

    dev = device if device is not None else rowptr.device
    counts = torch.tensor([rowptr.numel() - 1, col.numel()], dtype=torch.int64, device=dev)
    allc = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(allc, counts)
    rows = [int(c[0]) for c in allc]
    nnzs = [int(c[1]) for c in allc]
    if rank != 0:
        ops = [dist.P2POp(dist.isend, rowptr.contiguous(), 0)]
        if nnzs[rank]:
            ops += [dist.P2POp(dist.isend, col.contiguous(), 0), dist.P2POp(dist.isend, val.contiguous(), 0)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return None
    M, NNZ = sum(rows), sum(nnzs)
    out_rp = torch.zeros(M + 1, dtype=torch.int32, device=dev)
    out_ci = torch.empty(NNZ, dtype=col.dtype, device=dev)
    out_v = torch.empty(NNZ, dtype=val.dtype, device=dev)
    recv_rp = [None] * world
    ops = []
    for r in range(1, world):
        recv_rp[r] = torch.empty(rows[r] + 1, dtype=torch.int32, device=dev)
        ops.append(dist.P2POp(dist.irecv, recv_rp[r], r))
        if nnzs[r]:
            o = sum(nnzs[:r])
            ops.append(dist.P2POp(dist.irecv, out_ci[o:o + nnzs[r]], r))
            ops.append(dist.P2POp(dist.irecv, out_v[o:o + nnzs[r]], r))
    reqs = dist.batch_isend_irecv(ops) if ops else []
    out_ci[:nnzs[0]] = col
    out_v[:nnzs[0]] = val
    recv_rp[0] = rowptr
    for w in reqs:
        w.wait()
    ro, no = 0, 0
    for r in range(world):
        out_rp[ro:ro + rows[r] + 1] = recv_rp[r].to(torch.int32) + no
        ro += rows[r]
        no += nnzs[r]
    return out_rp, out_ci, out_v


def row_pieces(cum, m, world, nsub):
    """Rows [0, m) cut into world * nsub consecutive pieces of ~equal
    intermediate products (cum: the products of the row prefixes, length m+1;
    +1 per row so that runs of empty rows still spread), at ROW granularity: a
    hub tile row's 16 rows may go to different ranks (the CSR path has no tile
    rows).  Piece j is rank j % world's piece of round j // world, so that the
    pieces of one round are consecutive in C.  Returns pieces[round][rank] =
    (r0, r1).  (A single row heavier than a piece stays whole: none of the
    BASELINE configs has one -- webbase's heaviest row is 65 K of its 69 M
    products, the mawi prefix's 10^7 of 1.5 * 10^9.)"""
    cum = np.asarray(cum, dtype=np.float64)
    npc = max(1, world * nsub)
    w = cum + np.arange(m + 1, dtype=np.float64)
    bounds = [0]
    for j in range(1, npc):
        b = int(np.searchsorted(w, w[-1] * j / npc, side="left"))
        bounds.append(min(m, max(bounds[-1], b)))
    bounds.append(m)
    return [[(bounds[s * world + r], bounds[s * world + r + 1]) for r in range(world)] for s in range(nsub)]


class RoundGather:
    """Gather of C to rank 0 in rounds, each overlapped with the next round's
    computation.  The rows are cut into world x nsub pieces (row_pieces): rank
    r computes piece (s, r) in round s and hands it to push(s, ..., nnz).

    Counts travel on the host, never through a device read-back: every rank
    already holds its piece's nnz(C) as a host integer (the SpGEMM call returns
    it), and one non-blocking all_gather of those integers per round runs on a
    separate host (gloo) group, `meta_group`.  The peers post their sends at
    once and go on computing; rank 0 waits only for the round's host counts
    (no device synchronisation), then posts the receives of the peers' pieces
    straight into the final C at their exact offsets (the earlier rounds'
    nonzeros + the round's earlier pieces) and copies its own piece there.

    No concatenation: C's columns and values are written once on rank 0.  The
    output arrays are sized from the gathered nnz counts -- grown (after the
    receives into the old arrays complete) only when a round's counts exceed
    the capacity -- and kept across reset() calls, so a repeated product
    (the bench's steps) allocates them once at exactly nnz(C).  The returned
    arrays are views of the first nnz(C) entries, valid until the next step.
    Point-to-point messages between a pair match in posting order (RCCL/NCCL
    P2P have no tags): every pair posts rounds in order."""

    def __init__(self, rank, world, pieces, capacity=0, device=None, meta_group=None):
        import torch
        import torch.distributed as dist
        self.t, self.d = torch, dist
        self.rank, self.world, self.pieces = rank, world, pieces
        self.dev = device
        self.meta = meta_group  # host group of the counts (None: the default group, which must be gloo)
        self.cap = 0
        self.out_ci = self.out_v = None
        self.reset()
        if rank == 0:
            m = pieces[-1][-1][1] if pieces else 0
            self.out_rp = torch.empty(m + 1, dtype=torch.int32, device=device)
            self.m = m
            self._grow(max(1, int(capacity)))

    def reset(self):
        """start a new gather (one step) on the same pieces; rank 0 keeps its arrays"""
        self.off = 0            # rank 0: nonzeros of the rounds gathered so far
        self.work = []          # (work handle(s), tensors kept alive)
        self.fix = []           # rank 0: (received row pointers, first row, offset)
        self.meta_work = []     # peers: the count all_gathers still in flight

    def _wait(self):
        for ws, _ in self.work:
            for w in ws:
                w.wait()
        self.work = []

    def _grow(self, need):
        """rank 0: output arrays of at least `need` nonzeros, the first `off` kept"""
        t = self.t
        if need <= self.cap:
            return
        self._wait()  # (receives still landing in the old arrays)
        ci = t.empty(need, dtype=t.int32, device=self.dev)
        v = t.empty(need, dtype=t.float64, device=self.dev)
        if self.cap and self.off:
            ci[:self.off] = self.out_ci[:self.off]
            v[:self.off] = self.out_v[:self.off]
        self.out_ci, self.out_v, self.cap = ci, v, need

    def push(self, s, rowptr, col, val, nnz=None):
        """this rank's piece of round s (its rows' CSR, row pointers from 0;
        `nnz` its host-side nonzero count, default col.numel())"""
        t, d = self.t, self.d
        k_own = int(col.numel() if nnz is None else nnz)
        n = t.tensor([k_own], dtype=t.int64)
        alln = [t.zeros(1, dtype=t.int64) for _ in range(self.world)]
        h = d.all_gather(alln, n, group=self.meta, async_op=True)
        if self.rank != 0:
            rp = rowptr.contiguous()
            ops = [d.P2POp(d.isend, rp, 0)]
            keep = [rp]
            if k_own:
                c, v = col[:k_own].contiguous(), val[:k_own].contiguous()
                ops += [d.P2POp(d.isend, c, 0), d.P2POp(d.isend, v, 0)]
                keep += [c, v]
            self.work.append((d.batch_isend_irecv(ops), keep))
            self.meta_work.append((h, alln))
            return
        h.wait()  # the round's host counts (waits for the peers' progress, not for a device)
        nn = [int(x[0]) for x in alln]
        self._grow(self.off + sum(nn))
        o = self.off
        ops, keep = [], []
        for r in range(self.world):
            r0, r1 = self.pieces[s][r]
            k = nn[r]
            if r == 0:
                self.out_rp[r0:r1 + 1] = rowptr.to(t.int32) + o
                if k:
                    self.out_ci[o:o + k] = col[:k]
                    self.out_v[o:o + k] = val[:k]
            else:
                rp = t.empty(r1 - r0 + 1, dtype=t.int32, device=self.dev)
                ops.append(d.P2POp(d.irecv, rp, r))
                keep.append(rp)
                self.fix.append((rp, r0, o))
                if k:
                    ops.append(d.P2POp(d.irecv, self.out_ci[o:o + k], r))
                    ops.append(d.P2POp(d.irecv, self.out_v[o:o + k], r))
            o += k
        self.off = o
        if ops:
            self.work.append((d.batch_isend_irecv(ops), keep))

    def finish(self):
        self._wait()
        for h, _ in self.meta_work:
            h.wait()
        self.meta_work = []
        if self.rank != 0:
            return None
        for rp, r0, o in self.fix:  # the peers' row pointers, rebased
            self.out_rp[r0:r0 + rp.numel()] = rp + o
        self.fix = []
        self.out_rp[self.m] = self.off
        return self.out_rp, self.out_ci[:self.off], self.out_v[:self.off]
