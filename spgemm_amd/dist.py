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


def sub_blocks(cum, r_lo, r_hi, nsub, tile_m):
    """Rows [r_lo, r_hi) as `nsub` consecutive tile-row-aligned sub-blocks of
    ~equal intermediate products (cum = nnzCub of the row prefixes); some may
    be empty.  Every rank computes every rank's split the same way."""
    cum = np.asarray(cum, dtype=np.int64)
    bounds = [r_lo]
    for s in range(1, nsub):
        tgt = cum[r_lo] + (cum[r_hi] - cum[r_lo]) * s / nsub
        b = int(np.searchsorted(cum, tgt, side="left")) // tile_m * tile_m
        bounds.append(min(r_hi, max(bounds[-1], b)))
    bounds.append(r_hi)
    return list(zip(bounds[:-1], bounds[1:]))


class StreamingGather:
    """Gather of C row blocks to rank 0 overlapped with their computation.

    Each rank computes its rows as sub-blocks (sub_blocks above) and hands
    each one to push() as soon as it is done: a peer posts non-blocking sends
    of its row pointers (whose last entry, nnz, sizes the rest) and then its
    columns and values, and goes on computing the next sub-block while they
    travel; rank 0 posts the row-pointer receive of every peer's next
    sub-block ahead, and after each of its own sub-blocks turns the arrived
    row pointers into the column / value receives.  Point-to-point messages
    between a pair match in posting order (RCCL/NCCL P2P have no tags), so
    every peer's sub-blocks are received in order.  finish() returns the
    concatenated CSR (rank 0's sub-blocks, then rank 1's, ...) on rank 0 and
    None elsewhere.  sub_rows[r] = the row counts of rank r's sub-blocks."""

    def __init__(self, rank, world, sub_rows, device=None):
        import torch
        import torch.distributed as dist
        self.t, self.d = torch, dist
        self.rank, self.world, self.sub_rows = rank, world, sub_rows
        self.dev = device
        self.mine = []       # rank 0: its own sub-blocks
        self.sends = []      # peers: (work handle, tensor) kept alive until finish
        self.rp = {}         # rank 0: (peer, s) -> row pointer tensor being received
        self.rp_work = {}
        self.arr = {}        # rank 0: (peer, s) -> (col, val)
        self.arr_work = []
        self.next_s = [0] * world  # rank 0: each peer's next sub-block to turn into array receives
        if rank == 0:
            for r in range(1, world):
                self._post_rp(r, 0)

    def _post_rp(self, r, s):
        if s >= len(self.sub_rows[r]):
            return
        buf = self.t.empty(self.sub_rows[r][s] + 1, dtype=self.t.int32, device=self.dev)
        self.rp[(r, s)] = buf
        self.rp_work[(r, s)] = self.d.irecv(buf, r)

    def _advance(self, upto):
        """rank 0: every peer's sub-blocks < upto: row pointers waited for,
        column / value receives posted, the next row-pointer receive posted."""
        for r in range(1, self.world):
            while self.next_s[r] < min(upto, len(self.sub_rows[r])):
                s = self.next_s[r]
                self.rp_work.pop((r, s)).wait()
                nnz = int(self.rp[(r, s)][-1].item())
                col = self.t.empty(nnz, dtype=self.t.int32, device=self.dev)
                val = self.t.empty(nnz, dtype=self.t.float64, device=self.dev)
                if nnz:
                    self.arr_work.append(self.d.irecv(col, r))
                    self.arr_work.append(self.d.irecv(val, r))
                self.arr[(r, s)] = (col, val)
                self.next_s[r] = s + 1
                self._post_rp(r, s + 1)

    def push(self, s, rowptr, col, val):
        """this rank's sub-block s (its rows' CSR; row pointers from 0)"""
        if self.rank != 0:
            rp = rowptr.contiguous()
            self.sends.append((self.d.isend(rp, 0), rp))
            if col.numel():
                c, v = col.contiguous(), val.contiguous()
                self.sends.append((self.d.isend(c, 0), c))
                self.sends.append((self.d.isend(v, 0), v))
            return
        self.mine.append((rowptr, col, val))
        self._advance(s + 1)  # (peers finish sub-block s about when rank 0 does)

    def finish(self):
        if self.rank != 0:
            for w, _ in self.sends:
                w.wait()
            self.sends = []
            return None
        self._advance(max(len(x) for x in self.sub_rows))
        for w in self.arr_work:
            w.wait()
        t = self.t
        parts = [(rp, c, v) for rp, c, v in self.mine]
        for r in range(1, self.world):
            parts += [(self.rp[(r, s)],) + self.arr[(r, s)] for s in range(len(self.sub_rows[r]))]
        M = sum(p[0].numel() - 1 for p in parts)
        NNZ = sum(p[1].numel() for p in parts)
        out_rp = t.empty(M + 1, dtype=t.int32, device=self.dev)
        ro, no = 0, 0
        for rp, c, v in parts:
            k = rp.numel() - 1
            out_rp[ro:ro + k + 1] = rp.to(t.int32) + no
            ro += k
            no += c.numel()
        out_rp[M] = no
        out_ci = t.cat([p[1] for p in parts]) if parts else t.empty(0, dtype=t.int32, device=self.dev)
        out_v = t.cat([p[2] for p in parts]) if parts else t.empty(0, dtype=t.float64, device=self.dev)
        return out_rp, out_ci, out_v
