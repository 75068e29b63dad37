// tsg_ctiles.hip -- the reference's tiled C laid onto a C tile structure from a
// column-sorted CSR C, for the host tile API (tsg_tilespgemm) at 16 x 16 tiles.
//
// Reference layout (src/tilespgemm-cuda.h:2749-2775, tile2csr.h:8-68): per C
// tile t (tile_ptr / tile_columnidx from step 1, empty tiles included)
//   tile_nnz[t]        exclusive prefix of the tiles' nonzeros (tile_nnz[numtile] = nnz(C))
//   tile_csr_Ptr[t][r] exclusive prefix of the tile's row counts (u16)
//   mask[t][r]         bit 15 - c of the tile's row r (MSB first, csr2tile.h:193-195)
//   tile_csr_Col[p]    local column c (u16), tile_csr_Value[p] -- row-major inside the tile
// C's CSR rows are sorted, so tile row i's nonzeros (rows 16i..16i+15) are the
// CSR range [rowptr[16i], rowptr[16i+16]) and every tile of that row starts at
// rowptr[16i] + the nonzeros of the row's earlier tiles: no global scan.  The
// tiled payload is the CSR range reordered from (row, tile, column) to (tile,
// row, column): a transpose of the tile row's (row, tile) runs, each of at most
// 16 entries.
//
// A workgroup per unit of <= CT_TC tiles of one tile row (k_ctiles below); no
// global scan, no sort, every nonzero read twice and written once, every tile's
// Ptr and mask (the empty tiles' zeros included) written once, coalesced.
#include "tsg_internal.h"
#include "tsg_dev_common.h"

namespace tsg {

namespace {
constexpr int CT_NT = 256, CT_NW = CT_NT / 64;
constexpr int CT_TC = 496;                  // tiles per unit (LDS: 8 workgroups per CU; 992 tiles at 512 threads: +3 % on webbase)
constexpr int CT_TPT = (CT_TC + CT_NT - 1) / CT_NT;  // tiles per thread in the tile phase
constexpr int CT_EPT = 4;                   // nonzeros per thread held in registers (8: 1.91 vs 1.81 ms on webbase)
constexpr int CT_EB = CT_EPT * CT_NT;       // ... a batch of the unit's nonzeros
}  // namespace

// Units: (tile row i, tiles [c0, c1)) -- a tile row's tiles cut into runs of
// CT_TC, so that a wide tile row (webbase: up to 26 K tile-pattern tiles) is
// spread over many workgroups.  ucnt[i] = tile row i's units.
__global__ __launch_bounds__(WG) void k_ct_count(const int *tptr, int tilem, int *ucnt) {
    for (int i = blockIdx.x * WG + threadIdx.x; i < tilem; i += gridDim.x * WG)
        ucnt[i] = (tptr[i + 1] - tptr[i] + CT_TC - 1) / CT_TC;
}
// the unit list (ubase = ucnt scanned): units[u] = (i, c0, c1); *nu = their number
__global__ __launch_bounds__(WG) void k_ct_fill(const int *tptr, int tilem, const int *ubase, int4 *units, int *nu) {
    for (int i = blockIdx.x * WG + threadIdx.x; i < tilem; i += gridDim.x * WG) {
        const int t0 = tptr[i], t1 = tptr[i + 1], u0 = ubase[i];
        for (int k = 0; t0 + k * CT_TC < t1; ++k)
            units[u0 + k] = make_int4(i, t0 + k * CT_TC, min(t1, t0 + (k + 1) * CT_TC), 0);
        if (i == tilem - 1) *nu = ubase[tilem];
    }
}
// ulo[16u + r]: where row r of unit u's tile row reaches the unit's first tile
// column (the row start for a tile row's first unit).  A thread per (unit,
// row): the binary searches run here, all independent, rather than on each
// unit workgroup's critical path.
__global__ __launch_bounds__(WG) void k_ct_bounds(int m, const int *Crp, const int *Ccol, const int *tptr,
                                                  const int *tcol, const int4 *units, const int *nu, int *ulo) {
    const long nx = 16L * *nu;
    for (long x = (long)blockIdx.x * WG + threadIdx.x; x < nx; x += (long)gridDim.x * WG) {
        const int4 un = units[x >> 4];
        const int row = min(16 * un.x + (int)(x & 15), m);
        const int b0 = Crp[row];
        ulo[x] = (un.y == tptr[un.x] || row == m) ? b0 : lower_bound_dev(Ccol, b0, Crp[row + 1], 16 * tcol[un.y]);
    }
}

// A workgroup per unit (tile row i = rows 16i..16i+15, tiles [c0, c1) with
// columns tcl[0..n)):
//   * row r's nonzeros in the unit's columns: [ulo[16u+r], the next unit's
//     ulo or the row end); the unit's first tile offset = rowptr[16i] + the
//     row nonzeros before the range (units are independent: no carry);
//   * the unit's nonzeros, flat over its 16 row segments, CT_EPT per thread in
//     registers (columns, values, rows; every load independent), in batches
//     past CT_EB;
//   * pass A: each nonzero's tile by a binary search of tcl in LDS (kept in
//     registers for pass B when the unit is one batch); the (tile, row) masks
//     by LDS atomicOr (bit 15 - c, the reference's mask);
//   * tile totals = popcounts of the mask words, a workgroup scan -> the tiles'
//     offsets; then a thread per tile, consecutive tiles on consecutive lanes:
//     tile_nnz, Ptr and mask (2 x 16 B each; zeros for the empty tiles);
//   * pass B: each nonzero to offset + Ptr[row] + its rank in the row's mask
//     word (the popcount of the mask bits of smaller columns: the CSR row is
//     column-sorted, a column appears once), local column and value.
__global__ __launch_bounds__(CT_NT) void k_ctiles(int m, const int *Crp, const int *Ccol, const double *Cval,
                                                  const int *tptr, const int *tcol, const int4 *units, const int *nu,
                                                  const int *ulo, int *tnnz, u16 *Ptr, u16 *mask, u16 *Col,
                                                  double *Val, int *fail) {
    __shared__ __align__(16) u32 mk[CT_TC * 8];  // per unit tile: 16 mask words, two per u32 (row 2j low)
    __shared__ int toff[CT_TC];
    __shared__ int tcl[CT_TC];
    __shared__ int rs[16], lo[16], fpre[17];
    __shared__ int red[CT_NW + 1];
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int u = blockIdx.x;
    if (u >= *nu) return;  // (the grid is an upper bound of the units)
    const int4 un = units[u];
    const int i = un.x, c0 = un.y, c1 = un.z, n = c1 - c0;
    const int r0 = 16 * i;
    if (tid < 16) {
        const int row = min(r0 + tid, m);
        rs[tid] = Crp[row];
        lo[tid] = ulo[16 * u + tid];
        fpre[tid + 1] = c1 == tptr[i + 1] ? Crp[min(row + 1, m)] : ulo[16 * (u + 1) + tid];  // (the end, for now)
    }
    for (int t = tid; t < n; t += CT_NT) tcl[t] = tcol[c0 + t];
    for (int w = tid; w < 8 * n; w += CT_NT) mk[w] = 0u;
    __syncthreads();
    if (wv == 0) {  // segment lengths scanned; the unit's first offset
        const int v = lane < 16 ? fpre[lane + 1] - lo[lane] : 0;
        const int skip = lane < 16 ? lo[lane] - rs[lane] : 0;
        const int inc = wave_incl_scan_dpp(v);
        const int sk = wave_last(wave_incl_scan_dpp(skip));
        if (lane < 16) fpre[lane + 1] = inc;  // (lane l: the inclusive prefix of segments 0..l)
        if (lane == 0) {
            fpre[0] = 0;
            red[CT_NW] = rs[0] + sk;
        }
    }
    __syncthreads();
    const int nflat = fpre[16], base = red[CT_NW];
    const int nbat = (nflat + CT_EB - 1) / CT_EB;  // (workgroup-uniform)
    int cc[CT_EPT], rr[CT_EPT];                    // a batch: columns (-1: none), rows, values
    double xv[CT_EPT];
    auto load_batch = [&](int bb) {
        int ee[CT_EPT];
#pragma unroll
        for (int k = 0; k < CT_EPT; ++k) {
            const int q = bb * CT_EB + k * CT_NT + tid;
            int r = 0;
#pragma unroll
            for (int d = 8; d > 0; d >>= 1) r = r + d <= 16 && fpre[r + d] <= q ? r + d : r;
            rr[k] = r;
            ee[k] = q < nflat ? lo[r] + q - fpre[r] : -1;
        }
#pragma unroll
        for (int k = 0; k < CT_EPT; ++k) {
            cc[k] = ee[k] >= 0 ? Ccol[ee[k]] : -1;
            xv[k] = ee[k] >= 0 ? Cval[ee[k]] : 0.0;
        }
    };
    // the unit tile of a column (tcl ascending; every nonzero's tile is there)
    auto tile_of = [&](int col) -> int {
        const int tc = col >> 4;
        int a = 0, len = n;
        while (len > 1) {
            const int half = len >> 1;
            a = tcl[a + half] <= tc ? a + half : a;
            len -= half;
        }
        return tcl[a] == tc ? a : -1;
    };
    if (nbat == 1) load_batch(0);
    int tk[CT_EPT];  // (one batch: each nonzero's unit tile, kept for pass B)
    // pass A: the masks
    for (int bb = 0; bb < nbat; ++bb) {  // (workgroup-uniform)
        if (nbat > 1) load_batch(bb);
#pragma unroll
        for (int k = 0; k < CT_EPT; ++k) {
            const int tl = cc[k] >= 0 ? tile_of(cc[k]) : -1;
            tk[k] = tl;
            if (tl >= 0)
                atomicOr(&mk[tl * 8 + (rr[k] >> 1)], (0x8000u >> (cc[k] & 15)) << (16 * (rr[k] & 1)));
            else if (cc[k] >= 0)
                atomicExch(fail, 1);  // (never expected: a nonzero outside step 1's tiles)
        }
    }
    __syncthreads();
    {  // tile totals (a thread's tiles consecutive), scanned into the offsets
        int tot[CT_TPT], sum = 0;
#pragma unroll
        for (int k = 0; k < CT_TPT; ++k) {
            const int t = tid * CT_TPT + k;
            tot[k] = 0;
            if (t < n) {
                const uint4 a = reinterpret_cast<const uint4 *>(mk)[2 * t];
                const uint4 b = reinterpret_cast<const uint4 *>(mk)[2 * t + 1];
                tot[k] = __popc(a.x) + __popc(a.y) + __popc(a.z) + __popc(a.w) + __popc(b.x) + __popc(b.y) +
                         __popc(b.z) + __popc(b.w);
            }
            sum += tot[k];
        }
        const int inc = wave_incl_scan_dpp(sum);
        if (lane == 63) red[wv] = inc;
        __syncthreads();
        int off = inc - sum + base;
#pragma unroll
        for (int w = 0; w < CT_NW; ++w) off += w < wv ? red[w] : 0;
#pragma unroll
        for (int k = 0; k < CT_TPT; ++k) {
            const int t = tid * CT_TPT + k;
            if (t < n) toff[t] = off;
            off += tot[k];
        }
    }
    __syncthreads();
    // tile_nnz, Ptr and mask, consecutive tiles on consecutive lanes
    for (int t = tid; t < n; t += CT_NT) {
        const uint4 a = reinterpret_cast<const uint4 *>(mk)[2 * t];
        const uint4 b = reinterpret_cast<const uint4 *>(mk)[2 * t + 1];
        const u32 w8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        u32 pp[8];
        int run = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int lo16 = __popc(w8[j] & 0xffffu);
            pp[j] = (u32)run | ((u32)(run + lo16) << 16);
            run += __popc(w8[j]);
        }
        tnnz[c0 + t] = toff[t];
        // (nontemporal: 4.35 GB of Ptr and masks on webbase, never re-read by the
        // call -- k_ctiles 1.80 -> 1.53 ms; plain stores left them to compete for L2
        // and did not overlap the rest of the kernel; nontemporal tile_nnz, Col or
        // Value stores measured no gain or slower)
        typedef unsigned int v4 __attribute__((ext_vector_type(4)));
        v4 *dp = reinterpret_cast<v4 *>(Ptr + (size_t)(c0 + t) * 16);
        __builtin_nontemporal_store(v4{pp[0], pp[1], pp[2], pp[3]}, dp);
        __builtin_nontemporal_store(v4{pp[4], pp[5], pp[6], pp[7]}, dp + 1);
        v4 *dm = reinterpret_cast<v4 *>(mask + (size_t)(c0 + t) * 16);
        __builtin_nontemporal_store(v4{a.x, a.y, a.z, a.w}, dm);
        __builtin_nontemporal_store(v4{b.x, b.y, b.z, b.w}, dm + 1);
    }
    // pass B: every nonzero to its place
    for (int bb = 0; bb < nbat; ++bb) {  // (workgroup-uniform)
        if (nbat > 1) load_batch(bb);
#pragma unroll
        for (int k = 0; k < CT_EPT; ++k) {
            const int tl = nbat == 1 ? tk[k] : cc[k] >= 0 ? tile_of(cc[k]) : -1;
            if (tl >= 0) {
                const int r = rr[k], c = cc[k] & 15;
                const uint4 a = reinterpret_cast<const uint4 *>(mk)[2 * tl];
                const uint4 b = reinterpret_cast<const uint4 *>(mk)[2 * tl + 1];
                const u32 w8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
                int ptr = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) ptr += 2 * j + 1 < r ? __popc(w8[j]) : (2 * j < r ? __popc(w8[j] & 0xffffu) : 0);
                const u32 w = (w8[r >> 1] >> (16 * (r & 1))) & 0xffffu;
                const int rank = __popc(w >> (16 - c));  // (the row's smaller columns in this tile)
                const int dst = toff[tl] + ptr + rank;
                Col[dst] = (u16)c;
                Val[dst] = xv[k];
            }
        }
    }
}

}  // namespace tsg

namespace tsg {

// C (16 x 16, step 1's tile structure: tile_ptr, tile_columnidx, numtile) gets
// tile_nnz, tile_csr_Ptr, mask, tile_csr_Col and tile_csr_Value from the CSR C
// Cc (rows column-sorted, every nonzero inside some C tile).  Queued only; an
// entry outside the structure (never expected) sets cx.pinned[8] at the
// caller's next synchronisation.
int dev_ctiles_from_csr(Context &cx, const tsg_dev_csr &Cc, tsg_dev_tiles &C, hipStream_t s) {
    if (C.tile_m != 16 || C.tile_n != 16 || Cc.m != C.m) return TSG_ERR_INVALID;
    const size_t nt1 = (size_t)C.numtile + 1;
    TSG_TRY(cx.get(&C.tile_nnz, nt1));
    TSG_TRY(cx.get(&C.tile_csr_Ptr, nt1 * 16));
    TSG_TRY(cx.get(&C.mask, nt1 * 16));
    TSG_TRY(cx.get(&C.tile_csr_Col, (size_t)Cc.nnz + 1));
    TSG_TRY(cx.get(&C.tile_csr_Value, (size_t)Cc.nnz + 1));
    C.nnz = Cc.nnz;
    int *fail = nullptr, *ubase = nullptr, *ulo = nullptr;
    int4 *units = nullptr;
    const long umax = (long)C.numtile / CT_TC + C.tilem + 1;  // (units: an upper bound)
    TSG_TRY(cx.get(&fail, 2));
    TSG_TRY(cx.get(&ubase, (size_t)C.tilem + 1));
    TSG_TRY(cx.get(&units, (size_t)umax));
    TSG_TRY(cx.get(&ulo, 16 * (size_t)umax + 16));
    TSG_HIP(hipMemsetAsync(fail, 0, 2 * sizeof(int), s));
    cx.pinned[9] = Cc.nnz;  // tile_nnz[numtile] = nnz(C)
    TSG_HIP(hipMemcpyAsync(C.tile_nnz + C.numtile, cx.pinned + 9, sizeof(int), hipMemcpyHostToDevice, s));
    if (C.tilem > 0 && C.numtile > 0) {
        k_ct_count<<<grid_for(C.tilem, WG, 4096), WG, 0, s>>>(C.tile_ptr, C.tilem, ubase);
        TSG_HIP(hipMemsetAsync(ubase + C.tilem, 0, sizeof(int), s));
        TSG_TRY(scan_exclusive_i32(cx, ubase, (long)C.tilem + 1, s));
        k_ct_fill<<<grid_for(C.tilem, WG, 4096), WG, 0, s>>>(C.tile_ptr, C.tilem, ubase, units, fail + 1);
        k_ct_bounds<<<grid_for(16 * umax, WG, 16384), WG, 0, s>>>(C.m, Cc.rowpointer, Cc.columnindex, C.tile_ptr,
                                                                  C.tile_columnidx, units, fail + 1, ulo);
        k_ctiles<<<(unsigned)umax, CT_NT, 0, s>>>(C.m, Cc.rowpointer, Cc.columnindex, Cc.value, C.tile_ptr,
                                                  C.tile_columnidx, units, fail + 1, ulo, C.tile_nnz, C.tile_csr_Ptr,
                                                  C.mask, C.tile_csr_Col, C.tile_csr_Value, fail);
    }
    else if (Cc.nnz > 0)
        TSG_HIP(hipMemsetAsync(fail, 1, 1, s));  // (nonzeros but no tiles to hold them)
    TSG_HIP(hipGetLastError());
    cx.pinned[8] = 0;
    TSG_HIP(hipMemcpyAsync(cx.pinned + 8, fail, sizeof(int), hipMemcpyDeviceToHost, s));
    cx.put(fail);  // (stream-ordered reuse: the copies above precede any later use)
    cx.put(ubase);
    cx.put(units);
    cx.put(ulo);
    return TSG_OK;
}

}  // namespace tsg
