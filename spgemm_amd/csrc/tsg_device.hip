// tsg_device.hip -- hand-written gfx950 (CDNA4, wave64) kernels of the TileSpGEMM
// hot path, plus their stream-ordered host launchers.
//
// Pipeline (reference semantics in brackets, paths under /root/reference/src):
//   csr2tile A     [csr2tile.h:205-277]   keys -> segmented sort per tile row -> count -> scan -> fill
//   csr2tile B     [csr2tile.h:279-506]   same per B tile row + tile-level transpose into CSC tile order
//   step 1         [tilespgemm-cuda.h:279-392, nsparse :1171-1438]
//                  C tile structure: per (A tile row, column window) an LDS bitmask SPA
//   step 2         [tilespgemm-cuda.h:394-773]
//                  per C-tile-row chunk: LDS row masks OR-ed from B tile masks (ds_or_b32),
//                  popcount -> tile nnz / Ptr; device-wide scan of tile nnz [:2598-2604]
//   step 3         [tilespgemm-cuda.h:1273-2218]
//                  per C-tile-row chunk: LDS fp64 accumulator addressed by mask popcount rank
//                  (ds_add_f64), coalesced write of Val/Col
//   tile2csr       [tile2csr.h:72-140]    wave per C tile row, 16 wave scans per 64 tiles
//
// Row-wise (Gustavson over tiles) instead of the reference's per-C-tile set
// intersection: every (A tile, B tile) product of a C tile row is enumerated once
// per chunk with a load-balanced expansion across the 256-thread workgroup.
#include "tsg_internal.h"
#include "tsg_dev_common.h"

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace tsg {

// TSG_ABLATE diagnostics bitmask (documented above dev_step1), read once
static int g_ablate = -1;
static int ablate_bits() {
    if (g_ablate < 0) g_ablate = getenv("TSG_ABLATE") ? atoi(getenv("TSG_ABLATE")) : 0;
    return g_ablate;
}

// ---------------------------------------------------------------------------
// device-wide exclusive scan (reduce -> scan partials -> apply), in place
// ---------------------------------------------------------------------------
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = WG * SCAN_ITEMS;  // 4096 elements per block
__device__ __forceinline__ int scan_pad(int i) { return i + (i >> 4); }

template <class T> __global__ __launch_bounds__(WG) void k_scan_reduce(const T *a, long n, T *part) {
    __shared__ T red[WAVES];
    long base = (long)blockIdx.x * SCAN_TILE;
    T s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        long i = base + k * WG + threadIdx.x;
        if (i < n) s += a[i];
    }
    T tot = block_sum(s, red);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

template <class T, class P = T>
__global__ __launch_bounds__(WG) void k_scan_apply(T *a, long n, const P *part) {
    __shared__ T tile[SCAN_TILE + SCAN_TILE / 16];
    __shared__ T red[WAVES];
    long base = (long)blockIdx.x * SCAN_TILE;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        int li = k * WG + threadIdx.x;
        long i = base + li;
        tile[scan_pad(li)] = (i < n) ? a[i] : T(0);
    }
    __syncthreads();
    T s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) s += tile[scan_pad(threadIdx.x * SCAN_ITEMS + k)];
    T tot;
    T off = block_excl_scan(s, &tot, red) + (part ? (T)part[blockIdx.x] : T(0));
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        int li = scan_pad(threadIdx.x * SCAN_ITEMS + k);
        T v = tile[li];
        tile[li] = off;
        off += v;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        int li = k * WG + threadIdx.x;
        long i = base + li;
        if (i < n) a[i] = tile[scan_pad(li)];
    }
}

template <class T> static int scan_exclusive(Context &cx, T *a, long n, hipStream_t s) {
    if (n <= 0) return TSG_OK;
    long nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (nb == 1) {
        k_scan_apply<T><<<1, WG, 0, s>>>(a, n, (const T *)nullptr);
        TSG_HIP(hipGetLastError());
        return TSG_OK;
    }
    // (a single-pass decoupled look-back scan measured slower here: 17 vs 15 us
    // for mc2depi's 1.7 M entries, 25 vs 17 us for webbase's 3.1 M -- the
    // inclusive prefix crosses HBM once per 64 tiles of look-back, and the
    // status array needs its own memset)
    T *part = nullptr;
    TSG_TRY(cx.get(&part, nb));
    k_scan_reduce<T><<<(unsigned)nb, WG, 0, s>>>(a, n, part);
    TSG_HIP(hipGetLastError());
    TSG_TRY(scan_exclusive(cx, part, nb, s));
    k_scan_apply<T><<<(unsigned)nb, WG, 0, s>>>(a, n, part);
    TSG_HIP(hipGetLastError());
    cx.put(part);
    return TSG_OK;
}

int scan_exclusive_i32(Context &cx, int *a, long n, hipStream_t s) { return scan_exclusive(cx, a, n, s); }

__global__ __launch_bounds__(WG) void k_scan_reduce_wide(const int *a, long n, long long *part) {
    __shared__ long long red[WAVES];
    const long base = (long)blockIdx.x * SCAN_TILE;
    long long s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        const long i = base + k * WG + threadIdx.x;
        if (i < n) s += a[i];
    }
    const long long tot = block_sum(s, red);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
    if (blockIdx.x == 0 && threadIdx.x == 0) part[gridDim.x] = 0;  // the "n+1 scan" slot of the partials
}

// int32 exclusive scan whose block partials run in int64: *total = the exact
// sum (read back synchronously); TSG_ERR_OVERFLOW, with `a` left unscanned,
// when it does not fit an int32 index (C tile counts, nnz(C)).
// Exclusive int32 scan whose int64 total is read back to the host.  The apply
// kernel is queued before the read (the host round trip overlaps it); a total
// past INT_MAX returns TSG_ERR_OVERFLOW (the scanned values are then invalid).
// `before_read` (optional) queues more work ahead of the read, and extra_d
// (optional) is read back into *extra_h by the same host synchronisation.
template <class Fn>
static int scan_i32_total_impl(Context &cx, int *a, long n, hipStream_t s, long long *total, Fn &&before_read,
                               const long long *extra_d, long long *extra_h) {
    *total = 0;
    long long *part = nullptr;
    long nb = 0;
    if (n > 0) {
        nb = (n + SCAN_TILE - 1) / SCAN_TILE;
        TSG_TRY(cx.get(&part, (size_t)nb + 1));
        k_scan_reduce_wide<<<(unsigned)nb, WG, 0, s>>>(a, n, part);
        TSG_HIP(hipGetLastError());
        TSG_TRY(scan_exclusive(cx, part, nb + 1, s));
        k_scan_apply<int, long long><<<(unsigned)nb, WG, 0, s>>>(a, n, part);
        TSG_HIP(hipGetLastError());
    }
    before_read();
    if (part) TSG_HIP(hipMemcpyAsync(cx.pinned64, part + nb, sizeof(long long), hipMemcpyDeviceToHost, s));
    if (extra_d) TSG_HIP(hipMemcpyAsync(cx.pinned64 + 1, extra_d, sizeof(long long), hipMemcpyDeviceToHost, s));
    if (part || extra_d) TSG_TRY(stream_wait(s));
    if (part) *total = cx.pinned64[0];
    if (extra_d) *extra_h = cx.pinned64[1];
    cx.put(part);
    return *total > 0x7fffffffll ? TSG_ERR_OVERFLOW : TSG_OK;
}
int scan_exclusive_i32_total(Context &cx, int *a, long n, hipStream_t s, long long *total) {
    return scan_i32_total_impl(cx, a, n, s, total, [] {}, nullptr, nullptr);
}
int scan_exclusive_i64(Context &cx, long long *a, long n, hipStream_t s) {
    return scan_exclusive(cx, a, n, s);
}

// ---------------------------------------------------------------------------
// segmented sort of u64 keys (keys unique inside a segment for the >4096 tier)
//   tier 1: len <= 16    one thread, insertion sort in LDS
//   tier 2: len <= 512   one wave, bitonic network in its LDS slice
//   tier 3: len <= 4096  one workgroup, bitonic network in LDS
//   tier 4: len  > 4096  one workgroup: 4096-chunks sorted in LDS, then each key
//                        placed by its rank (sum of lower_bounds over the chunks)
// ---------------------------------------------------------------------------
constexpr int SORT_T1 = 16, SORT_T2 = 512, SORT_T3 = 4096;

__global__ __launch_bounds__(WG) void k_sort_classify(const int *seg, int nseg, int *lists, int *counts) {
    const int lane = lane_id();
    const u64 below = (1ull << lane) - 1ull;
    for (long base = (long)blockIdx.x * WG; base < nseg; base += (long)gridDim.x * WG) {
        const long i = base + threadIdx.x;
        int tier = -1;
        if (i < nseg) {
            int len = seg[i + 1] - seg[i];
            if (len > 1) tier = len <= SORT_T1 ? 0 : len <= SORT_T2 ? 1 : len <= SORT_T3 ? 2 : 3;
        }
        // one atomic per (wave, tier) instead of one per segment on 4 hot words
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const u64 msk = __ballot(tier == t);
            if (!msk) continue;
            const int leader = __ffsll((long long)msk) - 1;
            int pos0 = 0;
            if (lane == leader) pos0 = atomicAdd(&counts[t], __popcll(msk));
            pos0 = __builtin_amdgcn_readlane(pos0, leader);
            if (tier == t) lists[(long)t * nseg + pos0 + __popcll(msk & below)] = (int)i;
        }
    }
}

__global__ __launch_bounds__(WG) void k_sort_t1(u64 *keys, const int *seg, const int *list, const int *count) {
    __shared__ u64 buf[WG * SORT_T1];
    const int n = *count;
    u64 *my = buf + threadIdx.x * SORT_T1;
    for (int j = blockIdx.x * WG + threadIdx.x; j < n; j += gridDim.x * WG) {
        int i = list[j];
        int s = seg[i], len = seg[i + 1] - s;
        for (int q = 0; q < len; ++q) {
            u64 k = keys[s + q];
            int r = q - 1;
            while (r >= 0 && my[r] > k) { my[r + 1] = my[r]; --r; }
            my[r + 1] = k;
        }
        for (int q = 0; q < len; ++q) keys[s + q] = my[q];
    }
}

__device__ __forceinline__ void bitonic_step(u64 *s, int P, int k, int j, int t0, int tstride) {
    for (int t = t0; t < (P >> 1); t += tstride) {
        int i = 2 * t - (t & (j - 1));
        int l = i + j;
        bool up = (i & k) == 0;
        u64 a = s[i], b = s[l];
        if ((a > b) == up) { s[i] = b; s[l] = a; }
    }
}

__global__ __launch_bounds__(WG) void k_sort_t2(u64 *keys, const int *seg, const int *list, const int *count) {
    __shared__ u64 buf[WAVES * SORT_T2];
    const int n = *count;
    const int lane = lane_id();
    u64 *s = buf + wave_id() * SORT_T2;
    const int gw = (blockIdx.x * WG + threadIdx.x) >> 6, nw = gridDim.x * WAVES;
    for (int j = gw; j < n; j += nw) {
        int i = list[j];
        int st = seg[i], len = seg[i + 1] - st;
        int P = 64;
        while (P < len) P <<= 1;
        for (int q = lane; q < P; q += 64) s[q] = q < len ? keys[st + q] : ~0ull;
        wave_lds_sync();
        for (int k = 2; k <= P; k <<= 1)
            for (int jj = k >> 1; jj > 0; jj >>= 1) {
                bitonic_step(s, P, k, jj, lane, 64);
                wave_lds_sync();
            }
        for (int q = lane; q < len; q += 64) keys[st + q] = s[q];
        wave_lds_sync();
    }
}

__device__ void block_bitonic_sort(u64 *s, int P) {
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            bitonic_step(s, P, k, j, threadIdx.x, WG);
            __syncthreads();
        }
}

__global__ __launch_bounds__(WG) void k_sort_t3(u64 *keys, const int *seg, const int *list, const int *count) {
    __shared__ u64 s[SORT_T3];
    const int n = *count;
    for (int j = blockIdx.x; j < n; j += gridDim.x) {
        int i = list[j];
        int st = seg[i], len = seg[i + 1] - st;
        int P = 64;
        while (P < len) P <<= 1;
        for (int q = threadIdx.x; q < P; q += WG) s[q] = q < len ? keys[st + q] : ~0ull;
        __syncthreads();
        block_bitonic_sort(s, P);
        for (int q = threadIdx.x; q < len; q += WG) keys[st + q] = s[q];
        __syncthreads();
    }
}

// tier 4 work items are (segment, 4096-chunk) pairs spread over the whole grid;
// each workgroup walks the (short) list of big segments to find its pair.
__device__ __forceinline__ bool t4_pair(const int *seg, const int *list, int n, long idx, int *st, int *len,
                                        int *c) {
    for (int j = 0; j < n; ++j) {
        const int sg = list[j];
        const int l = seg[sg + 1] - seg[sg];
        const long nch = (l + SORT_T3 - 1) / SORT_T3;
        if (idx < nch) {
            *st = seg[sg];
            *len = l;
            *c = (int)idx;
            return true;
        }
        idx -= nch;
    }
    return false;
}

__global__ __launch_bounds__(WG) void k_sort_t4_chunks(u64 *keys, const int *seg, const int *list, const int *count) {
    __shared__ u64 s[SORT_T3];
    const int n = *count;
    int st, len, c;
    for (long idx = blockIdx.x; t4_pair(seg, list, n, idx, &st, &len, &c); idx += gridDim.x) {
        const int cs = st + c * SORT_T3, cl = min(SORT_T3, len - c * SORT_T3);
        for (int q = threadIdx.x; q < SORT_T3; q += WG) s[q] = q < cl ? keys[cs + q] : ~0ull;
        __syncthreads();
        block_bitonic_sort(s, SORT_T3);
        for (int q = threadIdx.x; q < cl; q += WG) keys[cs + q] = s[q];
        __syncthreads();
    }
}

// place every key of a chunk at its rank in the merged segment (keys unique)
__global__ __launch_bounds__(WG) void k_sort_t4_place(const u64 *keys, u64 *tmp, const int *seg, const int *list,
                                                      const int *count) {
    const int n = *count;
    int st, len, c;
    for (long idx = blockIdx.x; t4_pair(seg, list, n, idx, &st, &len, &c); idx += gridDim.x) {
        const int nch = (len + SORT_T3 - 1) / SORT_T3;
        const int cs = st + c * SORT_T3, cl = min(SORT_T3, len - c * SORT_T3);
        for (int q = threadIdx.x; q < cl; q += WG) {
            const u64 k = keys[cs + q];
            long rank = q;
            for (int o = 0; o < nch; ++o) {
                if (o == c) continue;
                const int os = st + o * SORT_T3, ol = min(SORT_T3, len - o * SORT_T3);
                rank += lower_bound_dev(keys + os, 0, ol, k);
            }
            tmp[st + rank] = k;
        }
    }
}

__global__ __launch_bounds__(WG) void k_sort_t4_copy(u64 *keys, const u64 *tmp, const int *seg, const int *list,
                                                     const int *count) {
    const int n = *count;
    int st, len, c;
    for (long idx = blockIdx.x; t4_pair(seg, list, n, idx, &st, &len, &c); idx += gridDim.x) {
        const int cs = st + c * SORT_T3, cl = min(SORT_T3, len - c * SORT_T3);
        for (int q = threadIdx.x; q < cl; q += WG) keys[cs + q] = tmp[cs + q];
    }
}

int segmented_sort_u64(Context &cx, u64 *keys, const int *seg, int nseg, long total, hipStream_t s) {
    if (nseg <= 0 || total <= 1) return TSG_OK;
    int *lists = nullptr, *counts = nullptr;
    u64 *tmp = nullptr;
    TSG_TRY(cx.get(&lists, (size_t)4 * nseg));
    TSG_TRY(cx.get(&counts, 4));
    TSG_TRY(cx.get(&tmp, (size_t)total));
    TSG_HIP(hipMemsetAsync(counts, 0, 4 * sizeof(int), s));
    k_sort_classify<<<grid_for(nseg, WG, 4096), WG, 0, s>>>(seg, nseg, lists, counts);
    k_sort_t1<<<grid_for(nseg, WG, 2048), WG, 0, s>>>(keys, seg, lists, counts);
    k_sort_t2<<<grid_for(nseg, WAVES, 2048), WG, 0, s>>>(keys, seg, lists + nseg, counts + 1);
    k_sort_t3<<<grid_for(nseg, 1, 1024), WG, 0, s>>>(keys, seg, lists + 2L * nseg, counts + 2);
    const int g4 = grid_for(total / SORT_T3 + 1, 1, 1024);
    k_sort_t4_chunks<<<g4, WG, 0, s>>>(keys, seg, lists + 3L * nseg, counts + 3);
    k_sort_t4_place<<<g4, WG, 0, s>>>(keys, tmp, seg, lists + 3L * nseg, counts + 3);
    k_sort_t4_copy<<<g4, WG, 0, s>>>(keys, tmp, seg, lists + 3L * nseg, counts + 3);
    TSG_HIP(hipGetLastError());
    cx.put(lists);
    cx.put(counts);
    cx.put(tmp);
    return TSG_OK;
}

// ---------------------------------------------------------------------------
// small utility kernels
// ---------------------------------------------------------------------------
__global__ void k_strided_starts(const int *rowptr, int m, int stride, int nseg, int *seg) {
    for (int i = blockIdx.x * WG + threadIdx.x; i <= nseg; i += gridDim.x * WG)
        seg[i] = rowptr[min((long)i * stride, (long)m)];
}

__global__ void k_set_i32(int *p, int v) { *p = v; }
__global__ void k_set_i64(long long *p, long long v) { *p = v; }

__global__ __launch_bounds__(WG) void k_nnzcub(const int *colA, long nnzA, const int *rowptrB,
                                               u64 *out) {
    __shared__ u64 red[WAVES];
    u64 s = 0;
    for (long p = (long)blockIdx.x * WG + threadIdx.x; p < nnzA; p += (long)gridDim.x * WG) {
        int k = colA[p];
        s += (u64)(rowptrB[k + 1] - rowptrB[k]);
    }
    s = block_sum(s, red);
    if (threadIdx.x == 0 && s) atomicAdd(out, s);
}

int launch_nnzcub(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, u64 *d_out, hipStream_t s) {
    (void)cx;
    TSG_HIP(hipMemsetAsync(d_out, 0, sizeof(u64), s));
    if (A.nnz > 0)
        k_nnzcub<<<grid_for(A.nnz, WG * 8, 4096), WG, 0, s>>>(A.columnindex, A.nnz, B.rowpointer, d_out);
    TSG_HIP(hipGetLastError());
    return TSG_OK;
}

int read_i32(Context &cx, const int *d, int *h, hipStream_t s) {
    TSG_HIP(hipMemcpyAsync(cx.pinned, d, sizeof(int), hipMemcpyDeviceToHost, s));
    TSG_TRY(stream_wait(s));
    *h = cx.pinned[0];
    return TSG_OK;
}

int read_i64(Context &cx, const long long *d, long long *h, hipStream_t s) {
    TSG_HIP(hipMemcpyAsync(cx.pinned64, d, sizeof(long long), hipMemcpyDeviceToHost, s));
    TSG_TRY(stream_wait(s));
    *h = cx.pinned64[0];
    return TSG_OK;
}

// ---------------------------------------------------------------------------
// stable CSR transpose (matrix_transposition, src/utils.h:161-198):
// column histogram -> scan -> unordered scatter of (row<<32 | pos) -> per-column
// segmented sort restores the row-ordered (stable) insertion order.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_colcount(const int *col, long nnz, int *cnt) {
    for (long p = (long)blockIdx.x * WG + threadIdx.x; p < nnz; p += (long)gridDim.x * WG)
        atomicAdd(&cnt[col[p]], 1);
}

__global__ __launch_bounds__(WG) void k_scatter_rows(const int *rowptr, const int *col, int m,
                                                     const int *colptr, int *fill, u64 *keys) {
    for (int r = blockIdx.x * WG + threadIdx.x; r < m; r += gridDim.x * WG)
        for (int p = rowptr[r]; p < rowptr[r + 1]; ++p) {
            int c = col[p];
            int slot = colptr[c] + atomicAdd(&fill[c], 1);
            keys[slot] = ((u64)(u32)r << 32) | (u32)p;
        }
}

__global__ __launch_bounds__(WG) void k_transpose_finish(const u64 *keys, long nnz, const double *val,
                                                         int *rowidx, double *oval) {
    for (long q = (long)blockIdx.x * WG + threadIdx.x; q < nnz; q += (long)gridDim.x * WG) {
        u64 k = keys[q];
        rowidx[q] = (int)(k >> 32);
        if (val) oval[q] = val[(u32)k];
    }
}

int dev_transpose(Context &cx, const tsg_dev_csr &A, tsg_dev_csr &out, hipStream_t s) {
    out.m = A.n;
    out.n = A.m;
    out.nnz = A.nnz;
    TSG_TRY(cx.get(&out.rowpointer, (size_t)A.n + 1));
    TSG_TRY(cx.get(&out.columnindex, (size_t)A.nnz + 1));
    TSG_TRY(cx.get(&out.value, (size_t)A.nnz + 1));
    int *fill = nullptr;
    u64 *keys = nullptr;
    TSG_TRY(cx.get(&fill, (size_t)A.n + 1));
    TSG_TRY(cx.get(&keys, (size_t)A.nnz + 1));
    TSG_HIP(hipMemsetAsync(out.rowpointer, 0, ((size_t)A.n + 1) * sizeof(int), s));
    TSG_HIP(hipMemsetAsync(fill, 0, ((size_t)A.n + 1) * sizeof(int), s));
    if (A.nnz > 0)
        k_colcount<<<grid_for(A.nnz, WG * 4, 8192), WG, 0, s>>>(A.columnindex, A.nnz, out.rowpointer);
    TSG_TRY(scan_exclusive_i32(cx, out.rowpointer, (long)A.n + 1, s));
    if (A.m > 0)
        k_scatter_rows<<<grid_for(A.m, WG, 8192), WG, 0, s>>>(A.rowpointer, A.columnindex, A.m,
                                                              out.rowpointer, fill, keys);
    TSG_TRY(segmented_sort_u64(cx, keys, out.rowpointer, A.n, A.nnz, s));
    if (A.nnz > 0)
        k_transpose_finish<<<grid_for(A.nnz, WG * 4, 8192), WG, 0, s>>>(keys, A.nnz, A.value,
                                                                        out.columnindex, out.value);
    TSG_HIP(hipGetLastError());
    cx.put(fill);
    cx.put(keys);
    return TSG_OK;
}

// ---------------------------------------------------------------------------
// csr2tile.  Sort key of an entry inside its tile row (TR CSR rows):
//   tc:26 | lr:6 | lc:6 | lpos:26
// A (row-major payload, csr2tile.h:152-192): lc = 0 -> order (tc, lr, CSR pos)
// B (per-tile transposed payload, csr2tile.h:390-484): order (tc, lr, lc, CSR pos)
// The sorted order IS the payload order inside each tile row.
// ---------------------------------------------------------------------------
constexpr int K_TC = 38, K_LR = 32, K_LC = 26;
constexpr u64 LPOS_MASK = (1ull << 26) - 1;
__device__ __forceinline__ u32 key_tc(u64 k) { return (u32)(k >> K_TC); }
__device__ __forceinline__ int key_lr(u64 k) { return (int)((k >> K_LR) & 63); }
__device__ __forceinline__ int key_lpos(u64 k) { return (int)(k & LPOS_MASK); }

template <int TR, int TC, bool WITH_LC>
__global__ __launch_bounds__(WG) void k_c2t_keys(const int *rowptr, const int *col, int m, u64 *keys) {
    for (int R = blockIdx.x * WG + threadIdx.x; R < m; R += gridDim.x * WG) {
        int i = R / TR;
        int rs = rowptr[i * TR];
        u64 lr = (u64)(R - i * TR);
        for (int p = rowptr[R]; p < rowptr[R + 1]; ++p) {
            int c = col[p];
            u64 tc = (u64)(c / TC);
            u64 lc = WITH_LC ? (u64)(c % TC) : 0ull;
            keys[p] = (tc << K_TC) | (lr << K_LR) | (lc << K_LC) | (u64)(p - rs);
        }
    }
}

// number of distinct tile columns per tile row (wave per tile row)
__global__ __launch_bounds__(WG) void k_c2t_count(const u64 *keys, const int *seg, int nseg, int *U) {
    const int lane = lane_id();
    const int gw = (blockIdx.x * WG + threadIdx.x) >> 6, nw = gridDim.x * WAVES;
    for (int i = gw; i < nseg; i += nw) {
        int s = seg[i], e = seg[i + 1];
        int cnt = 0;
        for (int base = s; base < e; base += 64) {
            int p = base + lane;
            bool in = p < e;
            u32 tc = in ? key_tc(keys[p]) : 0u;
            u32 tcp = (in && p > s) ? key_tc(keys[p - 1]) : 0xffffffffu;
            cnt += __popcll(__ballot(in && tc != tcp));
        }
        if (lane == 0) U[i] = cnt;
    }
}

enum { FILL_A = 0, FILL_B_STRUCT = 1, FILL_B_PAYLOAD = 2 };

// Wave per tile row.  TR = rows per tile (Ptr entries per tile), TC = cols per
// tile (TC/16 mask words per row).  Writes tiles of this tile row directly at
// their final positions:
//   FILL_A:         tile_columnidx/rowidx/nnz(start) + Ptr + Col(r*TC+c) + Val + mask
//   FILL_B_STRUCT:  row-major tile_columnidx/rowidx + per-tile nnz (row-major order)
//   FILL_B_PAYLOAD: CSC-ordered Ptr + Col(c) + Val + mask (tile id via rm2csc)
template <int TR, int TC, int MODE>
__global__ __launch_bounds__(WG) void k_c2t_fill(const u64 *keys, const int *seg, int nseg, const int *col,
                                                 const double *val, const int *tile_ptr, int *tcol,
                                                 int *trow, int *tnnz, u16 *Ptr, u16 *Col, double *Val,
                                                 u16 *mask, const int *rm2csc, const int *csc_nnz,
                                                 u16 *rm_mask, int *rm_rowstart) {
    constexpr int MW = TC / 16;
    const int lane = lane_id();
    const int gw = (blockIdx.x * WG + threadIdx.x) >> 6, nw = gridDim.x * WAVES;
    for (int i = gw; i < nseg; i += nw) {
        const int s = seg[i], e = seg[i + 1];
        const int tbase = tile_ptr[i];
        int carry_u = -1, carry_first = -1;
        for (int base = s; base < e; base += 64) {
            const int p = base + lane;
            const bool in = p < e;
            u64 k = in ? keys[p] : 0ull;
            u64 kp = (in && p > s) ? keys[p - 1] : 0ull;
            u64 kn = (in && p + 1 < e) ? keys[p + 1] : 0ull;
            const u32 tc = key_tc(k);
            const int lr = key_lr(k);
            const bool nt = in && (p == s || key_tc(kp) != tc);
            const bool te = in && (p + 1 == e || key_tc(kn) != tc);
            const bool gs = in && (nt || key_lr(kp) != lr);
            int u = carry_u + wave_incl_scan(nt ? 1 : 0);
            int f = max(wave_incl_max(nt ? p : -1), carry_first);
            carry_u = wave_last(u);
            carry_first = wave_last(f);
            if (!in) continue;
            const int trm = tbase + u;
            if (MODE == FILL_B_STRUCT) {
                if (nt) { tcol[trm] = (int)tc; trow[trm] = i; }
                if (te) tnnz[trm] = p - f + 1;
                continue;
            }
            const int t = (MODE == FILL_B_PAYLOAD) ? rm2csc[trm] : trm;
            const int src = s + key_lpos(k);
            const int c = col[src];
            const int lc = c % TC;
            const int dst = (MODE == FILL_B_PAYLOAD) ? csc_nnz[t] + (p - f) : p;
            Col[dst] = (MODE == FILL_A) ? (u16)(lr * TC + lc) : (u16)lc;
            Val[dst] = val[src];
            if (MODE == FILL_A && nt) {
                tcol[t] = (int)tc;
                trow[t] = i;
                tnnz[t] = p;
            }
            u16 *Pt = Ptr + (size_t)t * TR;
            u16 *Mt = mask + (size_t)t * TR * MW;
            // B: row-major views for the SpGEMM steps (no rm->csc indirection there)
            u16 *Mr = (MODE == FILL_B_PAYLOAD) ? rm_mask + (size_t)trm * TR * MW : nullptr;
            int *Rs = (MODE == FILL_B_PAYLOAD) ? rm_rowstart + (size_t)trm * (TR + 1) : nullptr;
            const int rsbase = (MODE == FILL_B_PAYLOAD) ? csc_nnz[t] : 0;
            if (gs) {
                const int rprev = nt ? -1 : key_lr(kp);
                for (int rr = rprev + 1; rr <= lr; ++rr) {
                    Pt[rr] = (u16)(p - f);
                    if (MODE == FILL_B_PAYLOAD) Rs[rr] = rsbase + (p - f);
                }
                for (int rr = rprev + 1; rr < lr; ++rr)
                    for (int w = 0; w < MW; ++w) {
                        Mt[rr * MW + w] = 0;
                        if (MODE == FILL_B_PAYLOAD) Mr[rr * MW + w] = 0;
                    }
                u16 mw[MW];
                for (int w = 0; w < MW; ++w) mw[w] = 0;
                for (int q = p; q < e; ++q) {
                    u64 kq = keys[q];
                    if (key_tc(kq) != tc || key_lr(kq) != lr) break;
                    int lcq = col[s + key_lpos(kq)] % TC;
                    mw[lcq >> 4] |= (u16)(1u << (15 - (lcq & 15)));
                }
                for (int w = 0; w < MW; ++w) {
                    Mt[lr * MW + w] = mw[w];
                    if (MODE == FILL_B_PAYLOAD) Mr[lr * MW + w] = mw[w];
                }
            }
            if (te) {
                for (int rr = lr + 1; rr < TR; ++rr) {
                    Pt[rr] = (u16)(p - f + 1);
                    if (MODE == FILL_B_PAYLOAD) Rs[rr] = rsbase + (p - f + 1);
                    for (int w = 0; w < MW; ++w) {
                        Mt[rr * MW + w] = 0;
                        if (MODE == FILL_B_PAYLOAD) Mr[rr * MW + w] = 0;
                    }
                }
                if (MODE == FILL_B_PAYLOAD) Rs[TR] = rsbase + (p - f + 1);
            }
        }
    }
}

// tile-level transpose of B's row-major tiles into CSC tile order
__global__ __launch_bounds__(WG) void k_tiles_colcount(const int *tcol, int numtile, int *cnt) {
    for (int t = blockIdx.x * WG + threadIdx.x; t < numtile; t += gridDim.x * WG) atomicAdd(&cnt[tcol[t]], 1);
}

__global__ __launch_bounds__(WG) void k_tiles_scatter(const int *tcol, const int *trow, int numtile,
                                                      const int *cptr, int *fill, u64 *keys) {
    for (int t = blockIdx.x * WG + threadIdx.x; t < numtile; t += gridDim.x * WG) {
        int c = tcol[t];
        int slot = cptr[c] + atomicAdd(&fill[c], 1);
        keys[slot] = ((u64)(u32)trow[t] << 32) | (u32)t;
    }
}

__global__ __launch_bounds__(WG) void k_tiles_finish(const u64 *keys, int numtile, int *csc_rowidx,
                                                     int *rm2csc, const int *nnz_rm, int *nnz_csc) {
    for (int q = blockIdx.x * WG + threadIdx.x; q < numtile; q += gridDim.x * WG) {
        u64 k = keys[q];
        int t = (int)(u32)k;
        csc_rowidx[q] = (int)(k >> 32);
        rm2csc[t] = q;
        nnz_csc[q] = nnz_rm[t];
    }
}

template <int TR, int TC>
static int csr2tile_impl(Context &cx, const tsg_dev_csr &M, bool colmajor, tsg_dev_tiles &out,
                         hipStream_t s) {
    const int m = M.m, n = M.n, nnz = M.nnz;
    const int tilem = (m + TR - 1) / TR, tilen = (n + TC - 1) / TC;
    if ((long)tilen >= (1L << 26)) return TSG_ERR_UNSUPPORTED;
    out = tsg_dev_tiles{};
    out.m = m; out.n = n; out.nnz = nnz;
    out.tile_m = TR; out.tile_n = TC;
    out.tilem = tilem; out.tilen = tilen;
    int *seg = nullptr, *U = nullptr;
    u64 *keys = nullptr;
    TSG_TRY(cx.get(&seg, (size_t)tilem + 1));
    TSG_TRY(cx.get(&keys, (size_t)nnz + 1));
    TSG_TRY(cx.get(&out.tile_ptr, (size_t)tilem + 1));
    k_strided_starts<<<grid_for(tilem + 1, WG, 4096), WG, 0, s>>>(M.rowpointer, m, TR, tilem, seg);
    if (m > 0) {
        if (colmajor)
            k_c2t_keys<TR, TC, true><<<grid_for(m, WG, 8192), WG, 0, s>>>(M.rowpointer, M.columnindex, m, keys);
        else
            k_c2t_keys<TR, TC, false><<<grid_for(m, WG, 8192), WG, 0, s>>>(M.rowpointer, M.columnindex, m, keys);
    }
    TSG_HIP(hipGetLastError());
    TSG_TRY(segmented_sort_u64(cx, keys, seg, tilem, nnz, s));
    U = out.tile_ptr;
    TSG_HIP(hipMemsetAsync(U, 0, ((size_t)tilem + 1) * sizeof(int), s));
    k_c2t_count<<<grid_for(tilem, WAVES, 8192), WG, 0, s>>>(keys, seg, tilem, U);
    TSG_HIP(hipGetLastError());
    TSG_TRY(scan_exclusive_i32(cx, out.tile_ptr, (long)tilem + 1, s));
    int numtile = 0;
    TSG_TRY(read_i32(cx, out.tile_ptr + tilem, &numtile, s));
    out.numtile = numtile;
    const size_t nt1 = (size_t)numtile + 1;
    TSG_TRY(cx.get(&out.tile_columnidx, nt1));
    TSG_TRY(cx.get(&out.tile_rowidx, nt1));
    TSG_TRY(cx.get(&out.tile_nnz, nt1));
    TSG_TRY(cx.get(&out.tile_csr_Ptr, nt1 * TR));
    TSG_TRY(cx.get(&out.tile_csr_Col, (size_t)nnz + 1));
    TSG_TRY(cx.get(&out.tile_csr_Value, (size_t)nnz + 1));
    TSG_TRY(cx.get(&out.mask, nt1 * TR * (TC / 16)));
    const int gfill = grid_for(tilem, WAVES, 8192);
    if (!colmajor) {
        k_c2t_fill<TR, TC, FILL_A><<<gfill, WG, 0, s>>>(keys, seg, tilem, M.columnindex, M.value, out.tile_ptr,
                                                       out.tile_columnidx, out.tile_rowidx, out.tile_nnz,
                                                       out.tile_csr_Ptr, out.tile_csr_Col, out.tile_csr_Value,
                                                       out.mask, nullptr, nullptr, nullptr, nullptr);
        k_set_i32<<<1, 1, 0, s>>>(out.tile_nnz + numtile, nnz);
        TSG_HIP(hipGetLastError());
    } else {
        int *nnz_rm = nullptr, *fill = nullptr;
        u64 *tkeys = nullptr;
        TSG_TRY(cx.get(&nnz_rm, nt1));
        TSG_TRY(cx.get(&fill, (size_t)tilen + 1));
        TSG_TRY(cx.get(&tkeys, nt1));
        TSG_TRY(cx.get(&out.csc_tile_ptr, (size_t)tilen + 1));
        TSG_TRY(cx.get(&out.csc_tile_rowidx, nt1));
        TSG_TRY(cx.get(&out.tile_rm2csc, nt1));
        TSG_TRY(cx.get(&out.rm_mask, nt1 * TR * (TC / 16)));
        TSG_TRY(cx.get(&out.rm_rowstart, nt1 * (TR + 1)));
        k_c2t_fill<TR, TC, FILL_B_STRUCT><<<gfill, WG, 0, s>>>(keys, seg, tilem, M.columnindex, M.value,
                                                              out.tile_ptr, out.tile_columnidx, out.tile_rowidx,
                                                              nnz_rm, nullptr, nullptr, nullptr, nullptr,
                                                              nullptr, nullptr, nullptr, nullptr);
        TSG_HIP(hipMemsetAsync(out.csc_tile_ptr, 0, ((size_t)tilen + 1) * sizeof(int), s));
        TSG_HIP(hipMemsetAsync(fill, 0, ((size_t)tilen + 1) * sizeof(int), s));
        if (numtile > 0)
            k_tiles_colcount<<<grid_for(numtile, WG, 8192), WG, 0, s>>>(out.tile_columnidx, numtile,
                                                                      out.csc_tile_ptr);
        TSG_TRY(scan_exclusive_i32(cx, out.csc_tile_ptr, (long)tilen + 1, s));
        if (numtile > 0)
            k_tiles_scatter<<<grid_for(numtile, WG, 8192), WG, 0, s>>>(out.tile_columnidx, out.tile_rowidx,
                                                                     numtile, out.csc_tile_ptr, fill, tkeys);
        TSG_TRY(segmented_sort_u64(cx, tkeys, out.csc_tile_ptr, tilen, numtile, s));
        if (numtile > 0)
            k_tiles_finish<<<grid_for(numtile, WG, 8192), WG, 0, s>>>(tkeys, numtile, out.csc_tile_rowidx,
                                                                    out.tile_rm2csc, nnz_rm, out.tile_nnz);
        k_set_i32<<<1, 1, 0, s>>>(out.tile_nnz + numtile, 0);
        TSG_TRY(scan_exclusive_i32(cx, out.tile_nnz, (long)numtile + 1, s));
        k_c2t_fill<TR, TC, FILL_B_PAYLOAD><<<gfill, WG, 0, s>>>(keys, seg, tilem, M.columnindex, M.value,
                                                               out.tile_ptr, nullptr, nullptr, nullptr,
                                                               out.tile_csr_Ptr, out.tile_csr_Col,
                                                               out.tile_csr_Value, out.mask, out.tile_rm2csc,
                                                               out.tile_nnz, out.rm_mask, out.rm_rowstart);
        TSG_HIP(hipGetLastError());
        cx.put(nnz_rm);
        cx.put(fill);
        cx.put(tkeys);
    }
    cx.put(seg);
    cx.put(keys);
    return TSG_OK;
}

// The SpGEMM steps are built for 16x16 tiles; csr2tile / tile2csr for every
// valid reference tile size with sides in {16, 32, 64}.
bool tile_size_supported(int tm, int tn) { return tm == 16 && tn == 16; }
bool tile_side_supported(int t) { return t == 16 || t == 32 || t == 48 || t == 64; }

template <int TR>
static int csr2tile_dispatch_c(Context &cx, const tsg_dev_csr &M, int tc, bool colmajor, tsg_dev_tiles &out,
                               hipStream_t s) {
    switch (tc) {
    case 16: return csr2tile_impl<TR, 16>(cx, M, colmajor, out, s);
    case 32: return csr2tile_impl<TR, 32>(cx, M, colmajor, out, s);
    case 48: return csr2tile_impl<TR, 48>(cx, M, colmajor, out, s);
    case 64: return csr2tile_impl<TR, 64>(cx, M, colmajor, out, s);
    default: return TSG_ERR_UNSUPPORTED;
    }
}

static int csr2tile_dispatch(Context &cx, const tsg_dev_csr &M, int tr, int tc, bool colmajor, tsg_dev_tiles &out,
                             hipStream_t s) {
    switch (tr) {
    case 16: return csr2tile_dispatch_c<16>(cx, M, tc, colmajor, out, s);
    case 32: return csr2tile_dispatch_c<32>(cx, M, tc, colmajor, out, s);
    case 48: return csr2tile_dispatch_c<48>(cx, M, tc, colmajor, out, s);
    case 64: return csr2tile_dispatch_c<64>(cx, M, tc, colmajor, out, s);
    default: return TSG_ERR_UNSUPPORTED;
    }
}

int dev_csr2tile_row_major(Context &cx, const tsg_dev_csr &A, int tm, int tn, tsg_dev_tiles &out,
                           hipStream_t s) {
    if (!tile_side_supported(tm) || !tile_side_supported(tn)) return TSG_ERR_UNSUPPORTED;
    return csr2tile_dispatch(cx, A, tm, tn, false, out, s);
}

int dev_csr2tile_col_major(Context &cx, const tsg_dev_csr &B, int tm, int tn, tsg_dev_tiles &out,
                           hipStream_t s) {
    if (!tile_side_supported(tm) || !tile_side_supported(tn)) return TSG_ERR_UNSUPPORTED;
    // B tiles are tn rows x tm cols
    return csr2tile_dispatch(cx, B, tn, tm, true, out, s);
}

// ---------------------------------------------------------------------------
// product enumeration: every (A tile a, B tile b) with a in A tile row [a0,a1)
// and b in B tile row colA[a] whose tile column lies in [clo, chi].  Items are
// spread over the 256 threads by an LDS exclusive scan of per-A-tile counts.
// ---------------------------------------------------------------------------
struct ProdLds {
    int bs[WG];
    int off[WG + 1];
    int red[WAVES];
};

// ebnd (optional): per A entry its B row's [start, end), one load instead of
// the colA -> bptr chain
template <class F>
__device__ __forceinline__ long for_each_product(int a0, int a1, const int *colA, const int *bptr,
                                                 const int *bcol, int clo, int chi, bool narrow,
                                                 ProdLds &L, F &&f, const int2 *ebnd = nullptr) {
    long items = 0;
    for (int ab = a0; ab < a1; ab += WG) {
        const int a = ab + threadIdx.x;
        int bs = 0, len = 0;
        if (a < a1) {
            int be;
            if (ebnd) {
                const int2 e = ebnd[a];
                bs = e.x;
                be = e.y;
            } else {
                int k = colA[a];
                bs = bptr[k];
                be = bptr[k + 1];
            }
            if (narrow) {
                bs = lower_bound_dev(bcol, bs, be, clo);
                be = lower_bound_dev(bcol, bs, be, chi + 1);
            }
            len = be - bs;
        }
        int tot;
        int off = block_excl_scan(len, &tot, L.red);
        L.bs[threadIdx.x] = bs;
        L.off[threadIdx.x] = off;
        __syncthreads();
        const int nA = min(WG, a1 - ab);
        for (int q = threadIdx.x; q < tot; q += WG) {
            const int lo = owner_search(L.off, nA, q);
            f(ab + lo, L.bs[lo] + (q - L.off[lo]));
        }
        items += tot;
        __syncthreads();
    }
    return items;
}

// Wave-sweep product enumeration (no per-product owner search): entries of the
// batch (thread t = entry ab + t) with a segment of <= WS_SHORT products walk
// it themselves; longer segments are compacted into an LDS list and swept by
// whole waves (lane l takes products bs + l, bs + l + 64, ...: coalesced B
// reads, wave-uniform entry).  f(a, b) for every product; returns this
// thread's share of the product count.
constexpr int WS_SHORT = 8;
struct WsLds {
    int2 seg[WG];   // long segments [bs, be)
    int ent[WG];    // their A entries
    int cnt[WAVES];
};
template <class F>
__device__ __forceinline__ long for_each_product_ws(int a0, int a1, const int2 *ebnd, const int *bcol, int clo,
                                                    int chi, bool narrow, WsLds &W, F &&f) {
    long items = 0;
    const int lane = lane_id(), wv = wave_id();
    for (int ab = a0; ab < a1; ab += WG) {
        const int a = ab + threadIdx.x;
        int bs = 0, be = 0;
        if (a < a1) {
            const int2 e = ebnd[a];
            bs = e.x;
            be = e.y;
            if (narrow) {
                bs = lower_bound_dev(bcol, bs, be, clo);
                be = lower_bound_dev(bcol, bs, be, chi + 1);
            }
        }
        items += be - bs;
        const bool lng = be - bs > WS_SHORT;
        if (!lng)
            for (int b = bs; b < be; ++b) f(a, b);
        const u64 m = __ballot(lng);
        if (lane == 0) W.cnt[wv] = __popcll(m);
        __syncthreads();
        int base = 0, total = 0;
#pragma unroll
        for (int w2 = 0; w2 < WAVES; ++w2) {
            const int v = W.cnt[w2];
            base += (w2 < wv) ? v : 0;
            total += v;
        }
        if (lng) {
            const int pos = base + __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
            W.seg[pos] = make_int2(bs, be);
            W.ent[pos] = a;
        }
        __syncthreads();
        for (int k = wv; k < total; k += WAVES) {  // wave-uniform
            const int2 sg = W.seg[k];
            const int ea = W.ent[k];
            for (int b = sg.x + lane; b < sg.y; b += 64) f(ea, b);
        }
        __syncthreads();  // the list is rewritten by the next batch
    }
    return items;
}

// ---------------------------------------------------------------------------
// step 1: C tile structure.  Unit = (A tile row i, window w of `win` B tile
// columns); an LDS bitmask collects the reachable tile columns.
//   PASS 0: count per unit (+ tile-product total); PASS 1: emit sorted columns.
// ---------------------------------------------------------------------------
constexpr int S1_MAXWORDS = 2048;  // 65536 tile columns per window

// thread t's wpt (1, 2, 4 or 8) consecutive bitmask words as vector LDS reads
// (scalar strided reads would put up to 8 lanes on one bank)
__device__ __forceinline__ void bm_words(const u32 *bm, int wpt, u32 *w) {
    const int t = threadIdx.x;
    if (wpt == 8) {
        const uint4 a = reinterpret_cast<const uint4 *>(bm)[2 * t], b = reinterpret_cast<const uint4 *>(bm)[2 * t + 1];
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    } else if (wpt == 4) {
        const uint4 a = reinterpret_cast<const uint4 *>(bm)[t];
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    } else if (wpt == 2) {
        const uint2 a = reinterpret_cast<const uint2 *>(bm)[t];
        w[0] = a.x; w[1] = a.y;
    } else {
        w[0] = bm[t];
    }
}

// Count (PASS 0) or emit (PASS 1) the set bits of bitmask words [wlo, whi]
// (bit b of word w = column clo + 32*w + b).  The full window goes through the
// vector reads; a narrower span (banded / local tile rows) touches only its
// own words, so clearing and scanning cost O(span), not O(window).
template <int PASS>
__device__ __forceinline__ void bm_count_emit(const u32 *bm, int words, int wpt, int wlo, int whi, int clo,
                                              int *red, int *unit_cnt, int u, int off0, int *out) {
    u32 wv[8];
    int base, nw;
    if (wlo == 0 && whi == words - 1) {
        bm_words(bm, wpt, wv);
        base = threadIdx.x * wpt;
        nw = wpt;
    } else {
        const int span = whi - wlo + 1, per = (span + WG - 1) / WG;
        base = wlo + threadIdx.x * per;
        nw = max(0, min(per, whi + 1 - base));
        for (int q = 0; q < 8; ++q) wv[q] = q < nw ? bm[base + q] : 0u;  // per <= 8 (span <= 2048)
    }
    int cnt = 0;
    for (int q = 0; q < nw; ++q) cnt += __popc(wv[q]);
    if (PASS == 0) {
        const int tot = block_sum(cnt, red);
        if (threadIdx.x == 0) unit_cnt[u] = tot;
    } else {
        int tot;
        int off = block_excl_scan(cnt, &tot, red) + off0;
        if (unit_cnt && threadIdx.x == 0) unit_cnt[u] = tot;  // emit into a unit buffer
        for (int q = 0; q < nw; ++q) {
            u32 x = wv[q];
            while (x) {
                out[off++] = clo + (base + q) * 32 + __ffs(x) - 1;
                x &= x - 1;
            }
        }
    }
}

//   PASS 0 with bm_store: the unit's bitmask is also stored (full window, vector
//   stores), and PASS 2 then emits from it instead of re-enumerating the tile
//   products (PASS 1).
// EL (CSR path, sparse tiles): the unit walks the ELEMENT products of CSR A's
// rows [16i, 16i+16) and CSR B's rows (Aptr = A row pointer, mA its row count,
// Bcol = B's element columns, bit = column / 16), so C gets only the tiles
// holding a nonzero -- for web-like matrices fewer products than the
// tile-pattern product, and no empty C tiles for steps 2 and 3.
//   PASS 0 with ubuf (EL): count AND emit the unit's sorted columns into its
//   slot ubuf[ubuf_off[u]..] (capacity = min(products, window)); k_step1_gather
//   then compacts the slots into tile_columnidx -- one element-product
//   enumeration instead of two.
template <int PASS, bool EL = false>
__global__ __launch_bounds__(WG) void k_step1(const int *Aptr, const int *Acol, const int *Bptr, const int *Bcol,
                                              int tilemA, int tilenB, int nwin, int win, int *unit_cnt,
                                              const int *unit_off, int *Ccol, u64 *prod_total, u32 *bm_store,
                                              int mA = 0, const int2 *ebnd = nullptr, int *ubuf = nullptr,
                                              const long long *ubuf_off = nullptr) {
    __shared__ __align__(16) u32 bm[S1_MAXWORDS];
    __shared__ ProdLds L;
    __shared__ WsLds W;
    __shared__ int red[WAVES];
    const int nunits = tilemA * nwin;
    const int words = win >> 5;
    const int wpt = words / WG;  // words per thread (win is a multiple of 8192)
    long my_items = 0;    // block totals (thread 0)
    long my_items_t = 0;  // per-thread shares (wave sweep)
    for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
        const int i = u / nwin, w = u - i * nwin;
        const int a0 = EL ? Aptr[min(i * 16, mA)] : Aptr[i], a1 = EL ? Aptr[min(i * 16 + 16, mA)] : Aptr[i + 1];
        if (a0 == a1) {
            if (PASS == 0 && threadIdx.x == 0) unit_cnt[u] = 0;
            continue;
        }
        const int clo = w * win, chi = min(clo + win, tilenB) - 1;
        if constexpr (PASS == 2) {
            const int o = unit_off[u], n = unit_off[u + 1] - o;
            if (n == 0) continue;  // uniform
            u32 wv[8];
            bm_words(bm_store + (size_t)u * words, wpt, wv);
            int cnt = 0;
            for (int q = 0; q < wpt; ++q) cnt += __popc(wv[q]);
            int tot;
            int off = block_excl_scan(cnt, &tot, red) + o;
            for (int q = 0; q < wpt; ++q) {
                u32 x = wv[q];
                while (x) {
                    Ccol[off++] = clo + (threadIdx.x * wpt + q) * 32 + __ffs(x) - 1;
                    x &= x - 1;
                }
            }
            continue;
        } else {
            const int wlo = 0, whi = words - 1;
            for (int q = wlo + threadIdx.x; q <= whi; q += WG) bm[q] = 0u;
            __syncthreads();
            auto mark = [&](int a, int b) {
                (void)a;
                int c = (EL ? Bcol[b] >> 4 : Bcol[b]) - clo;
                atomicOr(&bm[c >> 5], 1u << (c & 31));
            };
            if (EL) {
                my_items_t += for_each_product_ws(a0, a1, ebnd, Bcol, clo * 16, chi * 16 + 15, nwin > 1, W, mark);
            } else {
                long it = for_each_product(a0, a1, Acol, Bptr, Bcol, EL ? clo * 16 : clo, EL ? chi * 16 + 15 : chi,
                                           nwin > 1, L, mark, EL ? ebnd : nullptr);
                if (PASS == 0) my_items += (threadIdx.x == 0) ? it : 0;
            }
            if (PASS == 0 && bm_store) {
                u32 wv[8];
                bm_words(bm, wpt, wv);
                u32 *dst = bm_store + (size_t)u * words + threadIdx.x * wpt;
                for (int q = 0; q < wpt; q += 4) {
                    if (wpt >= 4) reinterpret_cast<uint4 *>(dst)[q / 4] = make_uint4(wv[q], wv[q + 1], wv[q + 2], wv[q + 3]);
                }
                if (wpt < 4)
                    for (int q = 0; q < wpt; ++q) dst[q] = wv[q];
            }
            if (PASS == 0 && ubuf)
                bm_count_emit<1>(bm, words, wpt, wlo, whi, clo, red, unit_cnt, u, 0, ubuf + ubuf_off[u]);
            else
                bm_count_emit<PASS>(bm, words, wpt, wlo, whi, clo, red, PASS == 1 ? nullptr : unit_cnt, u,
                                    PASS == 1 ? unit_off[u] : 0, Ccol);
            __syncthreads();
        }
    }
    if (PASS == 0 && EL) {
        my_items_t = wave_sum((long long)my_items_t);
        if (lane_id() == 0 && my_items_t) atomicAdd(prod_total, (u64)my_items_t);
    }
    if (PASS == 0 && threadIdx.x == 0 && my_items) atomicAdd(prod_total, (u64)my_items);
}

// EL step 1 unit-buffer capacities: wave per A tile row, its element products
// P (sum of its entries' B row lengths); every window of the row gets
// min(P, window width) slots.  With ciA / rpB it also fills the per-entry B
// row bounds ebnd (k_entry_bounds fused: the tile rows cover every entry once).
__global__ __launch_bounds__(WG) void k_step1_cap(const int *Aptr, int mA, int2 *ebnd, int tilemA, int nwin,
                                                  int win, int tilenB, long long *cap, const int *ciA,
                                                  const int *rpB, u64 *prod, int *ucnt) {
    const int lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // step 1's counters and the scans' n+1 slots
        const long nu = (long)tilemA * nwin;
        *prod = 0;
        ucnt[nu] = 0;
        cap[nu] = 0;
    }
    for (long i = ((long)blockIdx.x * WG + threadIdx.x) >> 6; i < tilemA; i += ((long)gridDim.x * WG) >> 6) {
        const int a0 = Aptr[min((int)i * 16, mA)], a1 = Aptr[min((int)i * 16 + 16, mA)];
        long long p = 0;
        for (int a = a0 + lane; a < a1; a += 64) {
            int2 e;
            if (ciA) {
                const int k = ciA[a];
                e = make_int2(rpB[k], rpB[k + 1]);
                ebnd[a] = e;
            } else {
                e = ebnd[a];
            }
            p += e.y - e.x;
        }
        p = wave_sum(p);
        for (int w = lane; w < nwin; w += 64)
            cap[i * nwin + w] = min(p, (long long)min(win, tilenB - w * win));
    }
}

// the same capacities at tile level (the tile-pattern step 1 of the host tile
// API): wave per A tile row, its tile products P = the B tile rows' lengths
// over its tiles; every window gets min(P, window width) slots
__global__ __launch_bounds__(WG) void k_step1_cap_tiles(const int *Atp, const int *Atc, const int *Btp, int tilemA,
                                                        int nwin, int win, int tilenB, long long *cap, u64 *prod,
                                                        int *ucnt) {
    const int lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // step 1's counters and the scans' n+1 slots
        const long nu = (long)tilemA * nwin;
        *prod = 0;
        ucnt[nu] = 0;
        cap[nu] = 0;
    }
    for (long i = ((long)blockIdx.x * WG + threadIdx.x) >> 6; i < tilemA; i += ((long)gridDim.x * WG) >> 6) {
        long long p = 0;
        for (int a = Atp[i] + lane; a < Atp[i + 1]; a += 64) {
            const int k = Atc[a];
            p += Btp[k + 1] - Btp[k];
        }
        p = wave_sum(p);
        for (int w = lane; w < nwin; w += 64)
            cap[i * nwin + w] = min(p, (long long)min(win, tilenB - w * win));
    }
}

// compact the step-1 unit buffers into tile_columnidx: a wave per unit (a
// unit holds ~1 K tile columns on webbase: a workgroup per unit left most of
// its lanes idle), four loads in flight per lane
__global__ __launch_bounds__(WG) void k_step1_gather(const int *ubuf, const long long *ubuf_off, const int *unit_off,
                                                     long nunits, int *Ccol) {
    const int lane = lane_id();
    for (long u = (long)blockIdx.x * WAVES + wave_id(); u < nunits; u += (long)gridDim.x * WAVES) {
        const int o = unit_off[u], n = unit_off[u + 1] - o;
        const int *src = ubuf + ubuf_off[u];
        int q = lane;
        for (; q + 192 < n; q += 256) {
            const int v0 = src[q], v1 = src[q + 64], v2 = src[q + 128], v3 = src[q + 192];
            Ccol[o + q] = v0;
            Ccol[o + q + 64] = v1;
            Ccol[o + q + 128] = v2;
            Ccol[o + q + 192] = v3;
        }
        for (; q < n; q += 64) Ccol[o + q] = src[q];
    }
}

__global__ void k_rows_from_units(const int *unit_off, int tilem, int nwin, int *Cptr) {
    for (int i = blockIdx.x * WG + threadIdx.x; i <= tilem; i += gridDim.x * WG) Cptr[i] = unit_off[(long)i * nwin];
}

// Tile structure only (tile_ptr + ascending distinct tile_columnidx per tile
// row) straight from CSR, the structural half of csr2tile (csr2tile.h:6-120):
// unit = (tile row i, window of `win` tile columns), LDS bitmask of the tile
// columns hit by the tile row's entries.  PASS 0 counts, PASS 1 emits.
//   flagged_only (PASS 0): only the units k_tcount16 marked -1
template <int PASS>
__global__ __launch_bounds__(WG) void k_tstruct(const int *rowptr, const int *col, int m, int tr, int tc, int tilem,
                                                int tilen, int nwin, int win, int *unit_cnt, const int *unit_off,
                                                int *tcol, int flagged_only = 0) {
    __shared__ __align__(16) u32 bm[S1_MAXWORDS];
    __shared__ int red[WAVES];
    __shared__ int red2[2 * WAVES];
    const int nunits = tilem * nwin;
    const int words = win >> 5;
    const int wpt = words / WG;
    for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
        if (PASS == 0 && flagged_only && unit_cnt[u] >= 0) continue;  // uniform
        const int i = u / nwin, w = u - i * nwin;
        const int p0 = rowptr[i * tr], p1 = rowptr[min((i + 1) * tr, m)];
        if (p0 == p1) {
            if (PASS == 0 && threadIdx.x == 0) unit_cnt[u] = 0;
            continue;
        }
        const int clo = w * win;
        int mn = 0x7fffffff, mx = -1;  // span of this window's tile columns
        for (int p = p0 + threadIdx.x; p < p1; p += WG) {
            const int c = col[p] / tc - clo;
            if ((unsigned)c < (unsigned)win) {
                mn = min(mn, c);
                mx = max(mx, c);
            }
        }
        block_minmax(mn, mx, red2);
        if (mx < mn) {
            if (PASS == 0 && threadIdx.x == 0) unit_cnt[u] = 0;
            continue;
        }
        int wlo = mn >> 5, whi = mx >> 5;
        if ((whi - wlo + 1) * 2 > words) wlo = 0, whi = words - 1;  // wide span: whole window, vector reads
        for (int x = wlo + threadIdx.x; x <= whi; x += WG) bm[x] = 0u;
        __syncthreads();
        for (int p = p0 + threadIdx.x; p < p1; p += WG) {
            const int c = col[p] / tc - clo;
            if ((unsigned)c < (unsigned)win) atomicOr(&bm[c >> 5], 1u << (c & 31));
        }
        __syncthreads();
        bm_count_emit<PASS>(bm, words, wpt, wlo, whi, clo, red, unit_cnt, u, PASS == 1 ? unit_off[u] : 0, tcol);
        __syncthreads();
    }
}

// Tile counts of 16x16 tile rows (one window), wave per tile row: the tile
// row's E <= 256 tile columns go into a wave-private LDS hash set (512 slots,
// linear probing, atomicCAS tells new from duplicate), so a tile row costs
// ~E/64 hash rounds and no workgroup syncs.  Larger tile rows get -1 and go to
// k_tstruct's bitmap.
constexpr int TC_SLOTS = 512;
__global__ __launch_bounds__(WG) void k_tcount16(const int *rowptr, const int *col, int m, int tilem, int *unit_cnt) {
    if (blockIdx.x == 0 && threadIdx.x == 0) unit_cnt[tilem] = 0;  // the scan's n+1 slot
    __shared__ __align__(16) u32 ht_all[WAVES * TC_SLOTS];
    u32 *ht = ht_all + wave_id() * TC_SLOTS;
    const int lane = lane_id();
    for (long i = ((long)blockIdx.x * WG + threadIdx.x) >> 6; i < tilem; i += ((long)gridDim.x * WG) >> 6) {
        const int p0 = rowptr[i * 16], p1 = rowptr[min((int)i * 16 + 16, m)];
        const int E = p1 - p0;
        if (E > TC_SLOTS / 2) {
            if (lane == 0) unit_cnt[i] = -1;
            continue;
        }
#pragma unroll
        for (int q = 0; q < TC_SLOTS / 256; ++q)
            reinterpret_cast<uint4 *>(ht)[q * 64 + lane] = make_uint4(~0u, ~0u, ~0u, ~0u);
        wave_lds_sync();
        int cnt = 0;
        for (int c = 0; c < E; c += 64) {
            bool fresh = false;
            if (c + lane < E) {
                const u32 tc = (u32)col[p0 + c + lane] >> 4;
                u32 h = (tc * 0x9E3779B1u) >> 23;  // 9 bits: TC_SLOTS = 512
                for (int pr = 0; pr < TC_SLOTS; ++pr) {
                    const u32 old = atomicCAS(&ht[h], ~0u, tc);
                    if (old == ~0u) { fresh = true; break; }
                    if (old == tc) break;
                    h = (h + 1) & (TC_SLOTS - 1);
                }
            }
            cnt += __popcll(__ballot(fresh));
        }
        wave_lds_sync();
        if (lane == 0) unit_cnt[i] = cnt;
    }
}

static void window_for(int tilen, int *win, int *nwin) {
    int w = 8192;  // power-of-two multiple of 8192 (1, 2, 4 or 8 bitmask words per thread)
    while (w < tilen && w < 65536) w <<= 1;
    *win = w;
    *nwin = (tilen + w - 1) / w;
}

// Row masks of a tiling straight from CSR (tile structure given): entry (R, c)
// sets bit 15 - c%16 of word (R % tr) * (tc/16) + (c % tc)/16 of its tile, the
// csr2tile mask layout (csr2tile.h:193-195).  mask must be zeroed.
__global__ __launch_bounds__(WG) void k_tile_masks(const int *rowptr, const int *col, int m, int tr, int tc,
                                                   const int *tile_ptr, const int *tcol, u16 *mask) {
    const int mw = tc / 16;
    u32 *m32 = reinterpret_cast<u32 *>(mask);
    for (int R = blockIdx.x * WG + threadIdx.x; R < m; R += gridDim.x * WG) {
        const int i = R / tr, r = R - i * tr;
        const int t0 = tile_ptr[i], t1 = tile_ptr[i + 1];
        for (int p = rowptr[R]; p < rowptr[R + 1]; ++p) {
            const int c = col[p];
            const int t = lower_bound_dev(tcol, t0, t1, c / tc);
            const int lc = c % tc;
            const long k = (long)t * tr * mw + r * mw + (lc >> 4);  // u16 index
            atomicOr(&m32[k >> 1], (0x8000u >> (lc & 15)) << ((k & 1) * 16));
        }
    }
}

int dev_tile_masks(Context &cx, const tsg_dev_csr &M, tsg_dev_tiles &t, u16 **mask_out, hipStream_t s) {
    const size_t words = ((size_t)t.numtile * t.tile_m * (t.tile_n / 16) + 2) & ~(size_t)1;
    TSG_TRY(cx.get(mask_out, words));
    TSG_HIP(hipMemsetAsync(*mask_out, 0, words * sizeof(u16), s));
    if (M.m > 0)
        k_tile_masks<<<grid_for(M.m, WG, 16384), WG, 0, s>>>(M.rowpointer, M.columnindex, M.m, t.tile_m, t.tile_n,
                                                             t.tile_ptr, t.tile_columnidx, *mask_out);
    TSG_HIP(hipGetLastError());
    return TSG_OK;
}

int dev_tile_structure(Context &cx, const tsg_dev_csr &M, int tr, int tc, tsg_dev_tiles &out, hipStream_t s,
                       double skip_emit_density) {
    out = tsg_dev_tiles{};
    out.m = M.m; out.n = M.n; out.nnz = M.nnz;
    out.tile_m = tr; out.tile_n = tc;
    out.tilem = (M.m + tr - 1) / tr;
    out.tilen = (M.n + tc - 1) / tc;
    int win, nwin;
    window_for(out.tilen, &win, &nwin);
    if ((long)out.tilem * nwin >= (1L << 31) - 1) return TSG_ERR_UNSUPPORTED;
    const long nunits = (long)out.tilem * nwin;
    int *ucnt = nullptr;
    TSG_TRY(cx.get(&ucnt, (size_t)nunits + 1));
    TSG_TRY(cx.get(&out.tile_ptr, (size_t)out.tilem + 1));
    const int g = grid_for(nunits, 1, 16384);
    const bool wave16 = out.tilem > 0 && tr == 16 && tc == 16 && nwin == 1 && !(ablate_bits() & 2048);
    if (!wave16) TSG_HIP(hipMemsetAsync(ucnt + nunits, 0, sizeof(int), s));  // (k_tcount16 zeroes it)
    if (out.tilem > 0) {
        if (wave16) {  // wave per tile row; the (rare) tile rows over 1024 entries then take the bitmap
            k_tcount16<<<grid_for((long)out.tilem * 64, WG, 16384), WG, 0, s>>>(M.rowpointer, M.columnindex, M.m,
                                                                               out.tilem, ucnt);
            k_tstruct<0><<<g, WG, 0, s>>>(M.rowpointer, M.columnindex, M.m, tr, tc, out.tilem, out.tilen, nwin, win,
                                          ucnt, nullptr, nullptr, 1);
        } else {
            k_tstruct<0><<<g, WG, 0, s>>>(M.rowpointer, M.columnindex, M.m, tr, tc, out.tilem, out.tilen, nwin, win,
                                          ucnt, nullptr, nullptr);
        }
    }
    TSG_HIP(hipGetLastError());
    TSG_TRY(scan_exclusive_i32(cx, ucnt, nunits + 1, s));
    k_rows_from_units<<<grid_for(out.tilem + 1, WG, 4096), WG, 0, s>>>(ucnt, out.tilem, nwin, out.tile_ptr);
    TSG_TRY(read_i32(cx, out.tile_ptr + out.tilem, &out.numtile, s));
    if ((double)M.nnz < skip_emit_density * (double)out.numtile) {  // caller needs the counts only
        cx.put(ucnt);
        return TSG_OK;
    }
    TSG_TRY(cx.get(&out.tile_columnidx, (size_t)out.numtile + 1));
    if (out.tilem > 0)
        k_tstruct<1><<<g, WG, 0, s>>>(M.rowpointer, M.columnindex, M.m, tr, tc, out.tilem, out.tilen, nwin, win,
                                      nullptr, ucnt, out.tile_columnidx);
    TSG_HIP(hipGetLastError());
    cx.put(ucnt);
    return TSG_OK;
}

// flag = 1 when some CSR row is not column-sorted (ascending, duplicates allowed)
// per unit: {e0, ei, esplit offset of its boundary row (lo, hi)} so step 2/3 can
// issue the split-point loads together with the unit's other loads
template <int TM>
__global__ void k_unit_etab(const int4 *utab, int nunits, const int *rpA, int m, const long long *ebase, int4 *etab) {
    for (int u = blockIdx.x * WG + threadIdx.x; u < nunits; u += gridDim.x * WG) {
        const int4 ut = utab[u];
        const int i = ut.x, q = ut.w >> 9;
        const int e0 = rpA[i * TM], ei = rpA[min((i + 1) * TM, m)] - e0;
        const long long off = ebase[i] + (long long)q * ei;
        etab[u] = make_int4(e0, ei, (int)(off & 0xffffffffll), (int)(off >> 32));
    }
}

// Element split points, one wave per unit (parallel over units x entries, no
// per-entry walk over all units of a hub row): entry x of the unit's tile row
// starts its segment at the first B row position reaching the unit's first
// tile column; the last unit also writes the row ends.
template <int TM>
__global__ __launch_bounds__(WG) void k_esplit_units(const int4 *utab, const int4 *etab, int nunits,
                                                     const int2 *ebnd, const int *ciB, const int *Ccol,
                                                     int *esplit) {
    const int lane = lane_id();
    for (int u = (blockIdx.x * WG + threadIdx.x) >> 6; u < nunits; u += gridDim.x * WAVES) {
        const int4 ut = utab[u], ue = etab[u];
        const int t0 = ut.y, nu = ut.z, q = ut.w >> 9;
        const int e0 = ue.x, ei = ue.y;
        int *sp = esplit + (((long long)(unsigned)ue.z) | ((long long)ue.w << 32));
        const int key = Ccol[t0] * TM;
        for (int x = lane; x < ei; x += 64) {
            const int2 b = ebnd[e0 + x];  // the entry's B row [b0, b1), one coalesced load
            sp[x] = q == 0 ? b.x : lower_bound_dev(ciB, b.x, b.y, key);
            if (q == nu - 1) sp[ei + x] = b.y;
        }
    }
}

// per A entry: its B row's position range
__global__ __launch_bounds__(WG) void k_entry_bounds(const int *ciA, long nnzA, const int *rpB, int2 *ebnd) {
    for (long p = (long)blockIdx.x * WG + threadIdx.x; p < nnzA; p += (long)gridDim.x * WG) {
        const int k = ciA[p];
        ebnd[p] = make_int2(rpB[k], rpB[k + 1]);
    }
}

// Row sortedness with no search: D = the non-ascents ci[p] <= ci[p-1] over
// all entries (a descent, or a column repeated), R = those at the first entry
// of a non-empty row (a thread per row).  The first entries of non-empty rows
// are distinct positions, so D - R counts the non-ascents inside rows: every
// row is strictly column-sorted iff D == R.  Each workgroup writes its share
// of D - R; one workgroup sums the shares and reports a nonzero total by a
// system-scope store into the caller's host-mapped flag.  (The shares of one
// workgroup do not cancel locally -- a row's first entry and the row itself
// sit in different workgroups -- and one atomic per workgroup on a common
// counter serialised: 47 us on mc2depi, 88 on webbase.)
constexpr int SRT_PT = 4;        // entries (and rows) per thread, their loads issued together
constexpr int SRT_MAXB = 4096;   // workgroups at most (grid-stride past it): few shares to sum
__global__ __launch_bounds__(WG) void k_rows_sorted_count(const int *rp, const int *ci, int m, int nnz, int *part) {
    __shared__ int red[WAVES];
    const int tid = threadIdx.x;
    const long n = max((long)nnz, (long)m);
    int v = 0;
    for (long b0 = (long)blockIdx.x * WG * SRT_PT; b0 < n; b0 += (long)gridDim.x * WG * SRT_PT) {
        int c0[SRT_PT], c1[SRT_PT], r0[SRT_PT], r1[SRT_PT];
#pragma unroll
        for (int u = 0; u < SRT_PT; ++u) {
            const long p = b0 + u * WG + tid;
            const bool okp = p >= 1 && p < nnz, okr = p < m;
            c0[u] = okp ? ci[p - 1] : 0;
            c1[u] = okp ? ci[p] : 1;
            r0[u] = okr ? rp[p] : 0;
            r1[u] = okr ? rp[p + 1] : 0;
        }
        int f0[SRT_PT], f1[SRT_PT];
#pragma unroll
        for (int u = 0; u < SRT_PT; ++u) {
            v += c1[u] <= c0[u];
            const bool st = r0[u] >= 1 && r0[u] < r1[u];  // a non-empty row past the first entry
            f0[u] = st ? ci[r0[u] - 1] : 0;
            f1[u] = st ? ci[r0[u]] : 1;
        }
#pragma unroll
        for (int u = 0; u < SRT_PT; ++u) v -= f1[u] <= f0[u];
    }
    v = block_sum(v, red);
    if (tid == 0) part[blockIdx.x] = v;
}
constexpr int SRT_FIN = 1024;  // the summing workgroup (mawi's 226 M rows: 2.2 * 10^5 shares)
__global__ __launch_bounds__(SRT_FIN) void k_rows_sorted_final(const int *part, int nb, int *hflag) {
    __shared__ long long red[SRT_FIN / 64];
    long long v = 0;
#pragma unroll 8
    for (int i = threadIdx.x; i < nb; i += SRT_FIN) v += part[i];
    v = wave_sum(v);
    if (lane_id() == 0) red[wave_id()] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
        for (int w = 0; w < SRT_FIN / 64; ++w) t += red[w];
        if (t != 0) __hip_atomic_store(hflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Queued only: the flag (1: some row is not column-sorted) lands in *host_flag
// (pinned, host-mapped: written by the kernel itself) by the caller's next
// stream synchronisation.
int dev_rows_sorted_shares(Context &cx, const tsg_dev_csr &M, int *host_flag, SortedShares *sh, hipStream_t s) {
    *host_flag = 0;
    *sh = SortedShares{};
    if (M.m > 0 && M.nnz > 1) {
        TSG_HIP(hipHostGetDevicePointer((void **)&sh->dflag, host_flag, 0));
        const long n = std::max<long>(M.nnz, M.m);
        const long nb = std::min<long>((n + WG * SRT_PT - 1) / (WG * SRT_PT), SRT_MAXB);
        TSG_TRY(cx.get(&sh->part, (size_t)nb));
        sh->nb = (int)nb;
        k_rows_sorted_count<<<(unsigned)nb, WG, 0, s>>>(M.rowpointer, M.columnindex, M.m, M.nnz, sh->part);
    }
    TSG_HIP(hipGetLastError());
    return TSG_OK;
}
// Sortedness of the B rows A references only (a row block of A against a far
// larger B: the mawi prefix reads ~7 K of B's 226 M rows, and the whole-B sweep
// above was 0.8 of its 4.1 ms).  k_ref_mark: a thread per A entry sets its B
// row's bit; the entry that set it first queues the row's chunks of SRT_CH
// adjacent pairs; k_ref_check: persistent workgroups over the queued chunks,
// each workgroup's count of non-ascents into its share.  The row-merge and band
// paths read only referenced rows, so this is the check they need; the staged
// tile pipeline reads whole B tile rows and gets the full check (the caller).
constexpr int SRT_CH = 4096;     // adjacent pairs per queued chunk of a long row (a workgroup's)
constexpr int SRT_SHORT = 64;    // rows of at most so many pairs: a thread's
constexpr int SRT_REFB = 1024;   // k_ref_check's workgroups (its shares)
__global__ __launch_bounds__(WG) void k_ref_mark(const int *ciA, int nnzA, const int *rpB, u32 *bits, int2 *items,
                                                 int *shorts, int *longs, int *cnt) {
    for (long a = (long)blockIdx.x * WG + threadIdx.x; a < nnzA; a += (long)gridDim.x * WG) {
        const int c = ciA[a];
        const u32 bit = 1u << (c & 31);
        if (atomicOr(&bits[c >> 5], bit) & bit) continue;  // (another entry queued the row)
        const int np = rpB[c + 1] - rpB[c] - 1;              // adjacent pairs
        if (np <= 0) continue;
        if (np <= SRT_SHORT) {
            shorts[atomicAdd(&cnt[1], 1)] = c;
            continue;
        }
        if (np <= SRT_CH) {
            items[atomicAdd(&cnt[0], 1)] = make_int2(c, 0);
            continue;
        }
        longs[atomicAdd(&cnt[2], 1)] = c;  // (its chunks spread over k_ref_check's workgroups: one
                                           // thread queueing the mawi hub's 2,441 chunks took 73 us)
    }
}
__global__ __launch_bounds__(WG) void k_ref_check(const int *rpB, const int *ciB, const int2 *items,
                                                  const int *shorts, const int *longs, const int *cnt, int *part) {
    __shared__ int red[WAVES];
    const int nl = cnt[0], ns = cnt[1], ng = cnt[2];
    int v = 0;
    for (int li = 0; li < ng; ++li) {  // (workgroup-uniform) rows past one chunk: chunk j on workgroup j mod grid
        const int c = longs[li];
        const int r0 = rpB[c], np = rpB[c + 1] - 1 - r0;
        for (int j = blockIdx.x; j * SRT_CH < np; j += gridDim.x) {
            const int p0 = r0 + j * SRT_CH, p1 = min(r0 + np, p0 + SRT_CH);
            for (int p = p0 + (int)threadIdx.x; p < p1; p += WG) v += ciB[p + 1] <= ciB[p];
        }
    }
    for (int q = blockIdx.x; q < nl; q += gridDim.x) {  // (workgroup-uniform) long rows' chunks
        const int2 it = items[q];
        const int p0 = rpB[it.x] + it.y * SRT_CH, p1 = min(rpB[it.x + 1] - 1, p0 + SRT_CH);
        for (int p = p0 + (int)threadIdx.x; p < p1; p += WG) v += ciB[p + 1] <= ciB[p];
    }
    for (int q = blockIdx.x * WG + threadIdx.x; q < ns; q += gridDim.x * WG) {  // short rows, a thread each
        const int c = shorts[q];
        const int p0 = rpB[c], p1 = rpB[c + 1] - 1;
        for (int p = p0; p < p1; p += 4) {  // (four pairs' loads at a time)
            int x[5];
#pragma unroll
            for (int u = 0; u < 5; ++u) x[u] = p + u <= p1 ? ciB[p + u] : INT_MAX;
#pragma unroll
            for (int u = 0; u < 4; ++u) v += p + u < p1 && x[u + 1] <= x[u];
        }
    }
    v = block_sum(v, red);
    if (threadIdx.x == 0) part[blockIdx.x] = v;
}
int dev_rows_sorted_shares_ref(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, int *host_flag,
                               SortedShares *sh, hipStream_t s) {
    *host_flag = 0;
    *sh = SortedShares{};
    if (B.m <= 0 || B.nnz <= 1 || A.nnz <= 0) return TSG_OK;
    TSG_HIP(hipHostGetDevicePointer((void **)&sh->dflag, host_flag, 0));
    u32 *bits = nullptr;
    int2 *items = nullptr;
    int *shorts = nullptr, *longs = nullptr;
    const size_t nw = ((size_t)B.m + 31) / 32;
    TSG_TRY(cx.get(&bits, nw + 3));  // (+3: the three queue counts after the bits)
    TSG_TRY(cx.get(&items, (size_t)A.nnz));
    TSG_TRY(cx.get(&shorts, (size_t)A.nnz));
    TSG_TRY(cx.get(&longs, (size_t)A.nnz));
    TSG_TRY(cx.get(&sh->part, (size_t)SRT_REFB));
    int *const cnt = reinterpret_cast<int *>(bits + nw);
    TSG_HIP(hipMemsetAsync(bits, 0, (nw + 3) * sizeof(u32), s));
    k_ref_mark<<<grid_for(A.nnz, WG, 16384), WG, 0, s>>>(A.columnindex, A.nnz, B.rowpointer, bits, items, shorts,
                                                          longs, cnt);
    k_ref_check<<<SRT_REFB, WG, 0, s>>>(B.rowpointer, B.columnindex, items, shorts, longs, cnt, sh->part);
    TSG_HIP(hipGetLastError());
    sh->nb = SRT_REFB;
    cx.put(bits);  // (stream-ordered reuse)
    cx.put(items);
    cx.put(shorts);
    cx.put(longs);
    return TSG_OK;
}
int dev_rows_sorted_finish(Context &cx, SortedShares &sh, hipStream_t s) {
    if (sh.part) {
        k_rows_sorted_final<<<1, SRT_FIN, 0, s>>>(sh.part, sh.nb, sh.dflag);
        cx.put(sh.part);  // (stream-ordered reuse)
    }
    sh = SortedShares{};
    TSG_HIP(hipGetLastError());
    return TSG_OK;
}
int dev_rows_sorted_async(Context &cx, const tsg_dev_csr &M, int *host_flag, hipStream_t s) {
    SortedShares sh;
    TSG_TRY(dev_rows_sorted_shares(cx, M, host_flag, &sh, s));
    return dev_rows_sorted_finish(cx, sh, s);
}
int dev_rows_sorted(Context &cx, const tsg_dev_csr &M, bool *sorted, hipStream_t s) {
    TSG_TRY(dev_rows_sorted_async(cx, M, cx.pinned + 1, s));
    TSG_TRY(stream_wait(s));
    *sorted = cx.pinned[1] == 0;
    return TSG_OK;
}

// ---------------------------------------------------------------------------
// Steps 2 and 3 share one chunking: unit = (C tile row i, <= CH consecutive C
// tiles of that row), units are independent workgroup tasks.  A unit's (A
// tile, B tile) products are the B tiles of each A tile's B row whose column
// lies in the unit's column range; they are spread item-by-item over the 256
// threads (consecutive items -> consecutive lanes, coalesced B reads).  Both
// steps OR the B tile row masks into LDS C row masks (the reference's step-2
// bitmask symbolic, tilespgemm-cuda.h:567-577); step 3 rebuilds them in LDS
// instead of round-tripping 32 B per C tile through HBM.  B is read through
// the row-major views (rm_mask, rm_rowstart) that csr2tile builds.
// ---------------------------------------------------------------------------
constexpr int CH = 256;          // C tiles per unit
#ifndef TSG_S3CAP
#define TSG_S3CAP 1024
#endif
#ifndef TSG_S3WPE
#define TSG_S3WPE 6
#endif
#ifndef TSG_GU_CAP
#define TSG_GU_CAP 65536  // measured: 16384 and 131072 both slower on webbase
#endif
#ifndef TSG_S2WPE
#define TSG_S2WPE 8
#endif
constexpr int S3_NZCAP = TSG_S3CAP;  // fp64 accumulator slots per numeric pass

template <int TM> struct CM {
    static constexpr int MW = TM / 16;           // u16 mask words per C row
    static constexpr int TW = TM * MW;           // u16 mask words per C tile
    static constexpr int TW32 = (TW + 1) / 2;    // u32 LDS words per C tile
};

template <int TM> __device__ __forceinline__ u32 lds_row_word(const u32 *tile, int r, int w) {
    const int k = r * CM<TM>::MW + w;
    return (tile[k >> 1] >> ((k & 1) * 16)) & 0xffffu;
}

struct ABView {
    const int *Aptr, *Acol, *Annz;
    const u16 *ColA;
    const double *ValA;
    const int *Bptr, *Bcol;
    const u16 *maskBrm;   // B tile masks, row-major tile order
    const int *rowsBrm;   // B tile absolute row starts (TN+1 per tile), row-major tile order
    const u16 *ColB;
    const double *ValB;
    const int *split;     // per (unit, A tile): first B tile of the unit's column range
    const long long *sbase;  // per C tile row: offset of its units' split entries
    const u16 *maskA;     // A tile masks (used when the A payload ColA/Annz is absent)
};

__global__ void k_units_per_row(const int *Cptr, int tilem, int *nunits) {
    for (int i = blockIdx.x * WG + threadIdx.x; i < tilem; i += gridDim.x * WG)
        nunits[i] = (Cptr[i + 1] - Cptr[i] + CH - 1) / CH;
    if (blockIdx.x == 0 && threadIdx.x == 0) nunits[tilem] = 0;
}

// unit -> C tile row (urow) and the unit table {i, t0, nu, q << 9 | ns} of step 3
// tbase (optional): the tile row's first C tile in another index space (the
// step-1 unit buffers, whose columns then need no compaction); t0 is then
// counted from tbase[i] instead of Cptr[i]
__global__ void k_unit_rows(const int *uoff, const int *Cptr, int tilem, int *urow, int4 *utab,
                            const long long *tbase) {
    for (int i = blockIdx.x * WG + threadIdx.x; i < tilem; i += gridDim.x * WG) {
        const int u0 = uoff[i], nu = uoff[i + 1] - u0, c0 = Cptr[i], c1 = Cptr[i + 1];
        const int b0 = tbase ? (int)tbase[i] : c0;
        for (int q = 0; q < nu; ++q) {
            urow[u0 + q] = i;
            const int t0 = c0 + q * CH;
            utab[u0 + q] = make_int4(i, b0 + q * CH, nu, (q << 9) | min(CH, c1 - t0));
        }
    }
}

// per (tile row, r): exclusive prefix of the unit row counts along the row's
// units (unit_rb) and the CSR row count (rowcnt)
template <int TM>
__global__ void k_unit_rowbase(const int *uoff, int tilem, int m, const int *unit_rc, int *unit_rb, int *rowcnt) {
    for (long x = (long)blockIdx.x * WG + threadIdx.x; x < (long)tilem * TM; x += (long)gridDim.x * WG) {
        const int i = (int)(x / TM), r = (int)(x - (long)i * TM);
        int run = 0;
        for (int u = uoff[i]; u < uoff[i + 1]; ++u) {
            const int v = unit_rc[(long)u * TM + r];
            unit_rb[(long)u * TM + r] = run;
            run += v;
        }
        if ((long)i * TM + r < m) rowcnt[(long)i * TM + r] = run;
    }
}

// tile row of every tile: one wave per tile row, coalesced stores (a thread per
// row serialised the long rows of C)
__global__ __launch_bounds__(WG) void k_crow(const int *Cptr, int tilem, int *Crow) {
    for (int i = blockIdx.x * WAVES + wave_id(); i < tilem; i += gridDim.x * WAVES)
        for (int t = Cptr[i] + lane_id(); t < Cptr[i + 1]; t += 64) Crow[t] = i;
}

// split entries per C tile row: (#units) x (#A tiles)
__global__ void k_split_counts(const int *uoff, const int *Aptr, int tilem, long long *sbase) {
    for (int i = blockIdx.x * WG + threadIdx.x; i < tilem; i += gridDim.x * WG)
        sbase[i] = (long long)(uoff[i + 1] - uoff[i]) * (Aptr[i + 1] - Aptr[i]);
    if (blockIdx.x == 0 && threadIdx.x == 0) sbase[tilem] = 0;
}

// first index in [lo, hi) with Bcol[idx] >= key (exponential search from lo)
__device__ __forceinline__ int gallop_ge(const int *Bcol, int lo, int hi, int key) {
    if (lo >= hi || Bcol[lo] >= key) return lo;
    int p = lo, step = 1;  // Bcol[p] < key
    while (p + step < hi && Bcol[p + step] < key) {
        p += step;
        step <<= 1;
    }
    int l = p + 1, h = min(p + step, hi);
    while (l < h) {
        const int mid = (l + h) >> 1;
        if (Bcol[mid] < key) l = mid + 1; else h = mid;
    }
    return l;
}

// thread per A tile: walk its B tile row once across the units of its C tile
// row, recording where each unit's column range starts
__global__ __launch_bounds__(WG) void k_unit_splits(int numtileA, const int *trowA, const int *Aptr, const int *Acol,
                                                    const int *Bptr, const int *Bcol, const int *uoff, const int *Cptr,
                                                    const int *Ccol, const long long *sbase, int *split) {
    for (int a = blockIdx.x * WG + threadIdx.x; a < numtileA; a += gridDim.x * WG) {
        const int i = trowA[a];
        const int lena = Aptr[i + 1] - Aptr[i], j = a - Aptr[i];
        const int nu = uoff[i + 1] - uoff[i];
        const int k = Acol[a];
        int p = Bptr[k];
        const int b1 = Bptr[k + 1];
        int *out = split + sbase[i] + j;
        for (int q = 0; q < nu; ++q) {
            if (q) p = gallop_ge(Bcol, p, b1, Ccol[Cptr[i] + q * CH]);
            out[(long)q * lena] = p;
        }
    }
}

// Element-streaming numeric: per (unit, A CSR entry of the C tile row) the
// first position in B's CSR row whose column reaches the unit's column range.
struct ECsr {
    int m;
    const int *rpA, *ciA;
    const double *vA;
    const int *rpB, *ciB;
    const double *vB;
    const int *esplit;
    const long long *ebase;
};

template <int TM>
__global__ void k_esplit_counts(const int *uoff, const int *rpA, int m, int tilem, long long *ebase) {
    for (int i = blockIdx.x * WG + threadIdx.x; i < tilem; i += gridDim.x * WG) {
        const int e0 = rpA[i * TM], e1 = rpA[min((long)(i + 1) * TM, (long)m)];
        ebase[i] = (long long)(uoff[i + 1] - uoff[i] + 1) * (e1 - e0);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) ebase[tilem] = 0;
}


// Products of A tiles [ab, ab+na) (row i, unit q of nu, A tiles from a0) that
// fall in the unit's column range, from the precomputed split points:
// bs[], off[] (exclusive scan of the counts, off[na] = total).
__device__ __forceinline__ int unit_setup(const ABView &V, int i, int q, int nu, int a0, int ab, int na, ProdLds &L) {
    const int a = ab + threadIdx.x;
    int bs = 0, len = 0;
    if (threadIdx.x < na) {
        const int lena = V.Aptr[i + 1] - a0;
        const int *sp = V.split + V.sbase[i] + (a - a0);
        bs = sp[(long)q * lena];
        const int be = (q + 1 < nu) ? sp[(long)(q + 1) * lena] : V.Bptr[V.Acol[a] + 1];
        len = be - bs;
    }
    int tot;
    const int off = block_excl_scan(len, &tot, L.red);
    L.bs[threadIdx.x] = bs;
    L.off[threadIdx.x] = off;
    if (threadIdx.x == 0) L.off[WG] = tot;
    __syncthreads();
    return tot;
}

// f(a, b, slot) for every item of the current setup
template <class F>
__device__ __forceinline__ void unit_items(const ABView &V, int ab, int na, int tot, const int *s_cols, int ns,
                                           ProdLds &L, F &&f) {
    for (int q = threadIdx.x; q < tot; q += WG) {
        const int lo = owner_search(L.off, na, q);
        const int b = L.bs[lo] + (q - L.off[lo]);
        f(ab + lo, b, lower_bound_u(s_cols, 0, ns, V.Bcol[b]));
    }
}

template <int TM, int TN>
__device__ __forceinline__ void or_product_masks(const ABView &V, int a, int b, u32 *tile) {
    constexpr int MW = CM<TM>::MW, AW = TN / 16;
    const u16 *mb = V.maskBrm + (size_t)b * TN * MW;
    if (!V.ColA) {  // A given by its tile masks: every set bit (r, c) ORs B row c into C row r
        const u16 *ma = V.maskA + (size_t)a * TM * AW;
        for (int r = 0; r < TM; ++r)
            for (int wa = 0; wa < AW; ++wa) {
                u32 bits = ma[r * AW + wa];
                while (bits) {
                    const int hb = 31 - __clz(bits);
                    const int c = wa * 16 + (15 - hb);
                    bits &= ~(1u << hb);
#pragma unroll
                    for (int w = 0; w < MW; ++w) {
                        const u32 mv = mb[c * MW + w];
                        if (mv) {
                            const int k = r * MW + w;
                            atomicOr(&tile[k >> 1], mv << ((k & 1) * 16));
                        }
                    }
                }
            }
        return;
    }
    const int q1 = V.Annz[a + 1];
    for (int qa = V.Annz[a]; qa < q1; ++qa) {
        const int enc = V.ColA[qa];
        const int r = enc / TN, c = enc - (enc / TN) * TN;
#pragma unroll
        for (int w = 0; w < MW; ++w) {
            const u32 mv = mb[c * MW + w];
            if (mv) {
                const int k = r * MW + w;
                atomicOr(&tile[k >> 1], mv << ((k & 1) * 16));
            }
        }
    }
}

template <int TM>
__device__ __forceinline__ void unit_load_cols_zero(const int *Ccol, int t0, int ns, int *s_cols, u32 *s_mask) {
    constexpr int TW32 = CM<TM>::TW32;
    for (int j = threadIdx.x; j < ns; j += WG) s_cols[j] = Ccol[t0 + j];
    uint4 *m4 = reinterpret_cast<uint4 *>(s_mask);
    const int n4 = (ns * TW32 + 3) / 4;
    for (int j = threadIdx.x; j < n4; j += WG) m4[j] = make_uint4(0u, 0u, 0u, 0u);
}

// OR the masks of every product of the unit.  Returns true when the whole
// row fitted one A batch, i.e. L still holds the setup for a second pass.
template <int TM, int TN>
__device__ __forceinline__ bool unit_masks(const ABView &V, int i, int q, int nu, int a0, int a1, const int *s_cols,
                                           int ns, u32 *s_mask, ProdLds &L, int *tot_out) {
    constexpr int TW32 = CM<TM>::TW32;
    int tot = 0;
    for (int ab = a0; ab < a1; ab += WG) {
        const int na = min(WG, a1 - ab);
        tot = unit_setup(V, i, q, nu, a0, ab, na, L);
        unit_items(V, ab, na, tot, s_cols, ns, L,
                   [&](int a, int b, int sl) { or_product_masks<TM, TN>(V, a, b, s_mask + sl * TW32); });
        __syncthreads();
    }
    *tot_out = tot;
    return a1 - a0 <= WG;
}

// ---------------------------------------------------------------------------
// step 2: per-tile nnz and per-unit per-row counts (-> CSR row pointers)
// ---------------------------------------------------------------------------
// Stream the element products of one unit straight from the CSR operands: for
// every A entry p of C tile row i (row r of the tile row) and every B entry pb
// of B row col(p) inside the unit's column range (split points precomputed by
// k_esplit_units; narrowed to columns [clo, chi) when `narrow`), call f(r, slot, pb),
// slot = p's index in the current batch of WG A entries (s_va[slot] = A value
// when s_va != nullptr).  Balanced over the workgroup by an LDS scan of the
// segment lengths (consecutive products -> consecutive lanes: coalesced B reads).
// first batch of a unit's element stream, loaded at the unit's start together
// with its masks (one dependent HBM round trip less per unit)
struct EPre {
    int bs, be;
    double va;
};

// Unit-table prefetch: a row (int4) fetched one int per lane (lanes 0..3), so it
// stays a divergent vector load whose wait sits at the row's first use
// (tab_row).  A uniform int4 load is compiled to a vector load followed at once
// by readfirstlane -- a full HBM round trip at the prefetch point.
__device__ __forceinline__ int tab_fetch(const int4 *tab, int u) {
    const int l = lane_id();
    return l < 4 ? reinterpret_cast<const int *>(tab + u)[l] : 0;
}
__device__ __forceinline__ int4 tab_row(int v) {
    return make_int4(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 1),
                     __builtin_amdgcn_readlane(v, 2), __builtin_amdgcn_readlane(v, 3));
}

__device__ __forceinline__ const int *etab_split(const ECsr &E, int4 ue) {
    return E.esplit + (((long long)(unsigned)ue.z) | ((long long)ue.w << 32));
}

__device__ __forceinline__ EPre epre_load(const ECsr &E, int4 ue, bool with_va) {
    EPre p{0, 0, 0.0};
    if ((int)threadIdx.x < ue.y) {
        const int *sp = etab_split(E, ue) + threadIdx.x;
        p.bs = sp[0];
        p.be = sp[ue.y];
        if (with_va) p.va = E.vA[ue.x + threadIdx.x];
    }
    return p;
}

// s_r: the A row (0..15) of each entry of a batch, in LDS (measured: int in
// step 2, u8 in step 3)
template <int TM, class SR, class F>
__device__ __forceinline__ void elem_stream(const ECsr &E, int4 ue, const EPre &pre, const int *s_rp, bool narrow,
                                            int clo, int chi, SR *s_r, double *s_va, ProdLds &L, F &&f) {
    const int e0 = ue.x, ei = ue.y;
    const int *sp0 = etab_split(E, ue);
    for (int eb = 0; eb < ei; eb += WG) {
        const int na = min(WG, ei - eb);
        int bs = 0, len = 0;
        if (threadIdx.x < na) {
            const int p = e0 + eb + threadIdx.x;
            int r = 0;  // last row of the tile row starting at or before entry p
#pragma unroll
            for (int st = TM / 2; st > 0; st >>= 1)
                if (s_rp[r + st] <= p) r += st;
            s_r[threadIdx.x] = (SR)r;
            int be;
            if (eb == 0) {
                bs = pre.bs;
                be = pre.be;
                if (s_va) s_va[threadIdx.x] = pre.va;
            } else {
                const int *sp = sp0 + (eb + threadIdx.x);
                bs = sp[0];
                be = sp[ei];
                if (s_va) s_va[threadIdx.x] = E.vA[p];
            }
            if (narrow) {
                bs = lower_bound_dev(E.ciB, bs, be, clo);
                be = lower_bound_dev(E.ciB, bs, be, chi);
            }
            len = be - bs;
        }
        int tot;
        const int off = block_excl_scan(len, &tot, L.red);
        L.bs[threadIdx.x] = bs;
        L.off[threadIdx.x] = off;
        __syncthreads();
        for (int it = threadIdx.x; it < tot; it += WG) {
            const int lo = owner_search(L.off, na, it);
            f((int)s_r[lo], lo, L.bs[lo] + (it - L.off[lo]));
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// step 2: C tile masks, per-tile nnz and per-unit per-row counts (-> CSR row
// pointers).  ELEM: masks from the CSR element products (sparse tiles);
// otherwise from the tile products (B row masks ORed per A nonzero).
// ---------------------------------------------------------------------------
// TSG_ABLATE & 64: per-phase shader-clock totals of k_step3 (thread 0 of each
// workgroup; diagnostics, printed by dev_tilespgemm)
// (compiled in only with -DTSG_PROF_BUILD)
__device__ unsigned long long g_prof[16];  // [0,8) step 3, [8,16) step 2
#ifdef TSG_PROF_BUILD
#define PROF_MARK(k)                                                         \
    if ((ablate & 64) && threadIdx.x == 0) {                                 \
        const u64 _t = __builtin_amdgcn_s_memtime();                         \
        atomicAdd(&g_prof[k], _t - prof_t);                                  \
        prof_t = _t;                                                         \
    }
#else
#define PROF_MARK(k)
#endif

template <int TM, int TN, bool ELEM>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(TSG_S2WPE))) void k_step2(const int4 *utab, const int4 *etab, int nunits, ABView V, ECsr E,
                                              const int *Ccol, int *nnzC, int *unit_rc, u16 *maskC, u16 *codeC,
                                              int ablate) {
#ifdef TSG_PROF_BUILD
    u64 prof_t = (ablate & 64) ? __builtin_amdgcn_s_memtime() : 0;
#endif
    constexpr int MW = CM<TM>::MW, TW32 = CM<TM>::TW32;
    __shared__ __align__(16) u32 s_mask[CH * TW32];
    __shared__ int s_cols[CH];
    __shared__ int s_rc[TM];
    __shared__ int s_rp[TM + 1];
    __shared__ int s_r[WG];
    __shared__ int s_wm[WAVES];
    __shared__ ProdLds L;
    // Software pipeline over this workgroup's units (stride G): the unit tables
    // run two units ahead and the unit's first loads (C tile columns, split
    // points, A row starts) one unit ahead, so the dependent HBM round trips of
    // a unit overlap the previous unit's work.
    struct UData {
        int col, rp;
        EPre pre;
    };
    const int G = gridDim.x;
    auto load_data = [&](int4 ut, int4 ue) {
        UData d{0, 0, {0, 0, 0.0}};
        const int t0 = ut.y, ns = ut.w & 511;
        if ((int)threadIdx.x < ns) d.col = Ccol[t0 + threadIdx.x];
        if (ELEM) {
            d.pre = epre_load(E, ue, false);
            if (threadIdx.x <= TM) d.rp = E.rpA[min(ut.x * TM + (int)threadIdx.x, E.m)];
        }
        return d;
    };
    constexpr bool LT = true;  // lane-fetched unit tables (tab_fetch)
    int4 ut_a = make_int4(0, 0, 0, 0), ue_a = ut_a, ut_b = ut_a, ue_b = ut_a;
    int tv_b = 0, ev_b = 0;  // tables of the unit two ahead (lanes 0..3, tab_fetch)
    UData d_a{0, 0, {0, 0, 0.0}};
    if ((int)blockIdx.x < nunits) {
        ut_a = utab[blockIdx.x];
        if (ELEM) ue_a = etab[blockIdx.x];
        d_a = load_data(ut_a, ue_a);
    }
    if ((int)blockIdx.x + G < nunits) {
        if (LT) {
            tv_b = tab_fetch(utab, blockIdx.x + G);
            if (ELEM) ev_b = tab_fetch(etab, blockIdx.x + G);
        } else {
            ut_b = utab[blockIdx.x + G];
            if (ELEM) ue_b = etab[blockIdx.x + G];
        }
    }
    for (int u = blockIdx.x; u < nunits; u += G) {
        const int4 ut = ut_a, ue = ue_a;
        const UData d = d_a;
        ut_a = LT ? tab_row(tv_b) : ut_b;
        if (ELEM) ue_a = LT ? tab_row(ev_b) : ue_b;
        if (u + G < nunits) d_a = load_data(ut_a, ue_a);
        if (u + 2 * G < nunits) {
            if (LT) {
                tv_b = tab_fetch(utab, u + 2 * G);
                if (ELEM) ev_b = tab_fetch(etab, u + 2 * G);
            } else {
                ut_b = utab[u + 2 * G];
                if (ELEM) ue_b = etab[u + 2 * G];
            }
        }
        const int i = ut.x, t0 = ut.y, nu = ut.z, q = ut.w >> 9, ns = ut.w & 511;
        const EPre pre = d.pre;
        if ((int)threadIdx.x < ns) s_cols[threadIdx.x] = d.col;
        {
            uint4 *m4 = reinterpret_cast<uint4 *>(s_mask);
            const int n4 = (ns * TW32 + 3) / 4;
            for (int x = threadIdx.x; x < n4; x += WG) m4[x] = make_uint4(0u, 0u, 0u, 0u);
        }
        if (threadIdx.x < TM) s_rc[threadIdx.x] = 0;
        if (ELEM && threadIdx.x <= TM) s_rp[threadIdx.x] = d.rp;
        __syncthreads();
        PROF_MARK(8);
        if (ELEM) {
            elem_stream<TM>(E, ue, pre, s_rp, false, 0, 0, s_r, nullptr, L, [&](int r, int, int pb) {
                const int x = E.ciB[pb];
                const int sl = lower_bound_u(s_cols, 0, ns, (int)((u32)x / TM));  // step 1 covers every product
                const int c = (int)((u32)x % TM), k = r * MW + (c >> 4);
                atomicOr(&s_mask[sl * TW32 + (k >> 1)], (0x8000u >> (c & 15)) << ((k & 1) * 16));
            });
        } else {
            int tot;
            unit_masks<TM, TN>(V, i, q, nu, V.Aptr[i], V.Aptr[i + 1], s_cols, ns, s_mask, L, &tot);
        }
        PROF_MARK(9);
        // row counts packed 4 x 16 bit (a unit's row count <= 256 * TM < 2^16)
        constexpr int NP = TM / 4;
        u64 pk[NP];
#pragma unroll
        for (int g = 0; g < NP; ++g) pk[g] = 0;
        static_assert((CM<TM>::TW32 % 4) == 0, "mask tile must be whole uint4");
        u32 w[TW32];  // tile j's words via vector LDS reads
        int nz = 0;
        const int j = threadIdx.x;
        if (j < ns) {  // ns <= CH == WG
#pragma unroll
            for (int k = 0; k < TW32 / 4; ++k) {
                const uint4 v = reinterpret_cast<const uint4 *>(s_mask + j * TW32)[k];
                w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
            }
#pragma unroll
            for (int r = 0; r < TM; ++r) {
                int c = 0;
#pragma unroll
                for (int ww = 0; ww < MW; ++ww) {
                    const int k = r * MW + ww;
                    c += __popc((w[k >> 1] >> ((k & 1) * 16)) & 0xffffu);
                }
                pk[r >> 2] += (u64)c << (16 * (r & 3));
                nz += c;
            }
            if (nnzC) nnzC[t0 + j] = nz;  // tile nnz (host tile API; the CSR path needs only row counts)
            if (!codeC) {  // C row masks in tile order (all-zero for empty tiles): the tile API's C.mask
                uint4 *dst = reinterpret_cast<uint4 *>(maskC + (size_t)(t0 + j) * CM<TM>::TW);
#pragma unroll
                for (int k = 0; k < TW32 / 4; ++k)
                    dst[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
            }
        }
        // wave totals per 32-bit half (no carries cross the 16-bit fields):
        // row r's count is field r & 1 of half r >> 1
        u32 hs[2 * NP];
#pragma unroll
        for (int h = 0; h < 2 * NP; ++h)
            hs[h] = (u32)__builtin_amdgcn_readlane(
                wave_incl_scan_dpp((int)(u32)(pk[h >> 1] >> (32 * (h & 1)))), 63);
        if (lane_id() < TM) {  // lane r adds row r's count of this wave
            u32 v = hs[0];
#pragma unroll
            for (int h = 1; h < 2 * NP; ++h) v = ((lane_id() >> 1) == h) ? hs[h] : v;
            const int c = (int)((v >> (16 * (lane_id() & 1))) & 0xffffu);
            if (c) atomicAdd(&s_rc[lane_id()], c);
        }
        u64 bm = 0;
        if (codeC) {
            bm = __ballot(nz > 1);
            if (lane_id() == 0) s_wm[wave_id()] = __popcll(bm);
        }
        __syncthreads();
        if (codeC && j < ns) {  // compact form for step 3 (16x16 tiles)
            u32 code = 0;
            if (nz == 1) {  // one nonzero: its in-tile position r << 4 | c
#pragma unroll
                for (int k = 0; k < TW32; ++k)
                    if (w[k]) {
                        const int hb = 31 - __clz(w[k]);
                        code = 0x8000u | (u32)((2 * k + (hb >> 4)) << 4) | (u32)(15 - (hb & 15));
                    }
            } else if (nz > 1) {  // full mask, compacted to the front of the unit's mask range
                int idx = __builtin_amdgcn_mbcnt_hi((u32)(bm >> 32), __builtin_amdgcn_mbcnt_lo((u32)bm, 0u));
                for (int w2 = 0; w2 < wave_id(); ++w2) idx += s_wm[w2];
                code = (u32)idx + 1;
                uint4 *dst = reinterpret_cast<uint4 *>(maskC + (size_t)(t0 + idx) * CM<TM>::TW);
#pragma unroll
                for (int k = 0; k < TW32 / 4; ++k)
                    dst[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
            }
            codeC[t0 + j] = (u16)code;
        }
        if (threadIdx.x < TM) unit_rc[(long)u * TM + threadIdx.x] = s_rc[threadIdx.x];
        __syncthreads();
        PROF_MARK(10);
    }
}

// ---------------------------------------------------------------------------
// step 3: numeric.  Per unit: masks rebuilt in LDS, then passes over tile
// sub-ranges holding <= S3_NZCAP nonzeros.  The LDS fp64 accumulator of a pass
// is in CSR order (row r, then tiles, then columns):
//   slot(s, r, x) = rowoff[r] + pre[s][r] + popc(row-r bits of columns < x)
// so the CSR epilogue (tile2csr fused) writes runs coalesced; the tile-layout
// output (Ptr/Col/Val, host API) is written per tile from the same slots.
// ---------------------------------------------------------------------------
template <int TM>
__device__ __forceinline__ int lds_rank(const u32 *tile, int r, int x) {
    constexpr int MW = CM<TM>::MW;
    int rank = 0;
#pragma unroll
    for (int w = 0; w < MW; ++w) {
        const u32 v = lds_row_word<TM>(tile, r, w);
        if (w < (x >> 4)) rank += __popc(v);
        else if (w == (x >> 4)) rank += __popc(v >> (16 - (x & 15)));
    }
    return rank;
}

// k-th (0-based) set column of a row word (MSB-first: bit 15-c = column c)
__device__ __forceinline__ int kth_col16(u32 v, int k) {
    u32 w = __brev(v) >> 16;  // bit c = column c
    for (int t = 0; t < k; ++t) w &= w - 1;
    return __ffs(w) - 1;
}


// rank of column c among row r's set bits plus all bits of rows < r
// (row-major in-tile position of (r, c); 16x16 tiles, MSB-first row words)
__device__ __forceinline__ int tile_rank16(const u32 *tile, int r, int c) {
    // two vector LDS reads, masked popcounts (no per-word branches)
    const uint4 a = reinterpret_cast<const uint4 *>(tile)[0], b = reinterpret_cast<const uint4 *>(tile)[1];
    const u32 wv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const int kr = r >> 1;
    int rank = 0;
    u32 row = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        rank += __popc(wv[k] & (k < kr ? ~0u : 0u));
        row = (k == kr) ? wv[k] : row;
    }
    if (r & 1) {
        rank += __popc(row & 0xffffu);
        row >>= 16;
    }
    return rank + __popc((row & 0xffffu) >> (16 - c));  // bits of columns < c (column c = bit 15 - c)
}

// Step 3 with a TILE-MAJOR accumulator: a pass's nonzeros sit at
// s_off[tile] - base + (row-major rank inside the tile), so the value pass needs
// only the tile offsets (one block scan of tile nnz) and the tile mask.  The
// CSR order across tiles is produced in the epilogue: every nonzero knows its
// row r, and its rank among the pass's row-r nonzeros in tile order comes from
// per-row ballots (16 per wave and 256 nonzeros) plus running per-row counters.
// RST (denser tiles): a per-tile table of row-start ranks (u8) in LDS replaces
// the eight popcounts of tile_rank16 on every product, at +4 KB of LDS.
template <int TM, int TN, bool WCSR, bool WTILE, bool ELEM, bool RST = false>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(RST ? 5 : TSG_S3WPE))) void k_step3(const int4 *utab, const int4 *etab, int nunits, int mrows, ABView V,
                                              ECsr E, const int *Ccol,
                                              const int *nnzoff, const u16 *maskC, const u16 *codeC,
                                              const int *unit_rb,
                                              const int *rowptr, int *csr_col, double *csr_val, u16 *PtrC,
                                              u16 *ColC, double *ValC, int ablate) {
    static_assert(TM == 16, "tile-major step 3 is built for 16x16 C tiles");
    constexpr int TW32 = CM<TM>::TW32, NV4 = TW32 / 4;
    static_assert(CH == WG, "one C tile per thread");
    __shared__ __align__(16) u32 s_mask[CH * TW32];
    __shared__ __align__(16) double acc[S3_NZCAP];
    __shared__ __align__(16) double s_va[WG];
    __shared__ int s_cols[CH];
    __shared__ int s_off[CH + 1];           // [j]: nonzeros of the unit's tiles [0, j)
    __shared__ int s_rp[TM + 1];            // A CSR row starts of the tile row (ELEM)
    __shared__ unsigned char s_r[WG];
    __shared__ unsigned char s_key[S3_NZCAP];  // pass nonzero e: r << 4 | c
    static_assert(CH <= 256, "a unit's tile index fits a byte");
    __shared__ unsigned char s_kt[S3_NZCAP];   // pass nonzero e: its tile
    __shared__ unsigned char s_rs[RST ? CH * TM : 1];  // [tile][r]: in-tile rank of row r's first nonzero
    __shared__ int s_wcnt[WAVES][TM];       // per-wave row counts of the current 256 nonzeros
    __shared__ int s_run[TM];               // row-r nonzeros of this pass already placed
    __shared__ int s_carry[TM];             // row-r nonzeros of this unit's earlier passes
    __shared__ int s_rowptr[TM];
    __shared__ int s_red[WAVES];
    __shared__ ProdLds L;
    const int j = threadIdx.x, lane = lane_id(), wv = wave_id();
#ifdef TSG_PROF_BUILD
    u64 prof_t = (ablate & 64) ? __builtin_amdgcn_s_memtime() : 0;
#endif
    // Software pipeline over this workgroup's units (stride G): the unit tables
    // run two units ahead, the tile codes one unit ahead, and the unit's inputs
    // (C masks + columns, row bases, first element batch) are issued for the
    // next unit once this unit's value pass is done, so their HBM round trip
    // overlaps this unit's CSR writes.
    const int G = gridDim.x;
    u32 nw[TW32];
    int ncol = 0, nrb = 0, nrw = 0, nrp = 0;
    EPre npre{0, 0, 0.0};
    auto issue = [&](int un, int4 utx, int4 uex, u32 cd) {
        const int t0x = utx.y, nsx = utx.w & 511, ix = utx.x;
#pragma unroll
        for (int k = 0; k < TW32; ++k) nw[k] = 0u;
        ncol = 0;
        if (j < nsx) {
            if (WCSR) {  // compact form (k_step2): 0 empty, 0x8000|pos one nonzero, idx+1 full mask
                if (cd & 0x8000u) {
                    const int r = (cd >> 4) & 15, c = cd & 15;
#pragma unroll
                    for (int k = 0; k < TW32; ++k) nw[k] = (k == (r >> 1)) ? (0x8000u >> c) << ((r & 1) * 16) : 0u;
                } else if (cd) {
                    const uint4 *src = reinterpret_cast<const uint4 *>(maskC + (size_t)(t0x + cd - 1) * CM<TM>::TW);
#pragma unroll
                    for (int k = 0; k < NV4; ++k) {
                        const uint4 v = src[k];
                        nw[4 * k] = v.x; nw[4 * k + 1] = v.y; nw[4 * k + 2] = v.z; nw[4 * k + 3] = v.w;
                    }
                }
            } else {
                const uint4 *src = reinterpret_cast<const uint4 *>(maskC + (size_t)(t0x + j) * CM<TM>::TW);
#pragma unroll
                for (int k = 0; k < NV4; ++k) {
                    const uint4 v = src[k];
                    nw[4 * k] = v.x; nw[4 * k + 1] = v.y; nw[4 * k + 2] = v.z; nw[4 * k + 3] = v.w;
                }
            }
            ncol = Ccol[t0x + j];
        }
        if (WCSR && j < TM) {
            nrb = unit_rb[(long)un * TM + j];
            nrw = rowptr[min(ix * TM + j, mrows)];
        }
        if (ELEM && j <= TM) nrp = E.rpA[min(ix * TM + j, E.m)];
        if (ELEM && !(ablate & 4)) npre = epre_load(E, uex, true);
    };
    constexpr bool LT = !RST;  // lane-fetched tables (measured: a loss for the few, long RST units)
    int4 ut_c = make_int4(0, 0, 0, 0), ue_c = ut_c, ut_n = ut_c, ue_n = ut_c;
    int tv_n = 0, ev_n = 0;  // tables of the unit two ahead (lanes 0..3, tab_fetch)
    u32 code_n = 0;
    if ((int)blockIdx.x < nunits) {
        ut_c = utab[blockIdx.x];
        if (ELEM) ue_c = etab[blockIdx.x];
        if (WCSR && j < (ut_c.w & 511)) code_n = codeC[ut_c.y + j];
        issue(blockIdx.x, ut_c, ue_c, code_n);
    }
    if ((int)blockIdx.x + G < nunits) {
        if (LT) {
            tv_n = tab_fetch(utab, blockIdx.x + G);
            if (ELEM) ev_n = tab_fetch(etab, blockIdx.x + G);
        } else {
            ut_n = utab[blockIdx.x + G];
            if (ELEM) ue_n = etab[blockIdx.x + G];
        }
    }
    for (int u = blockIdx.x; u < nunits; u += G) {
        PROF_MARK(7);
        const int4 ut = ut_c, ue = ue_c;
        ut_c = LT ? tab_row(tv_n) : ut_n;
        if (ELEM) ue_c = LT ? tab_row(ev_n) : ue_n;
        if (u + 2 * G < nunits) {
            if (LT) {
                tv_n = tab_fetch(utab, u + 2 * G);
                if (ELEM) ev_n = tab_fetch(etab, u + 2 * G);
            } else {
                ut_n = utab[u + 2 * G];
                if (ELEM) ue_n = etab[u + 2 * G];
            }
        }
        const bool more = u + G < nunits;
        const int i = ut.x, t0 = ut.y, nu = ut.z, q = ut.w >> 9, ns = ut.w & 511;
        const EPre pre = npre;
        u32 w[TW32];
#pragma unroll
        for (int k = 0; k < TW32; ++k) w[k] = nw[k];
        if (threadIdx.x < TM) {
            s_carry[threadIdx.x] = WCSR ? nrb : 0;
            if (WCSR) s_rowptr[threadIdx.x] = nrw;
        }
        if (ELEM && threadIdx.x <= TM) s_rp[threadIdx.x] = nrp;
#pragma unroll
        for (int k = 0; k < NV4; ++k)
            reinterpret_cast<uint4 *>(s_mask + j * TW32)[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2],
                                                                         w[4 * k + 3]);
        s_cols[j] = ncol;
        int tt = 0;
        if (RST) {
            u32 rs4[TM / 4];
#pragma unroll
            for (int r = 0; r < TM; ++r) {
                if ((r & 3) == 0) rs4[r >> 2] = 0;
                rs4[r >> 2] |= (u32)tt << (8 * (r & 3));
                tt += __popc((w[r >> 1] >> ((r & 1) * 16)) & 0xffffu);
            }
#pragma unroll
            for (int k = 0; k < TM / 16; ++k)
                reinterpret_cast<uint4 *>(s_rs + j * TM)[k] = make_uint4(rs4[4 * k], rs4[4 * k + 1], rs4[4 * k + 2],
                                                                         rs4[4 * k + 3]);
        } else {
#pragma unroll
            for (int k = 0; k < TW32; ++k) tt += __popc(w[k]);
        }
        int ttot;
        const int toff = block_excl_scan(tt, &ttot, s_red);
        s_off[j] = toff;
        if (j == WG - 1) s_off[CH] = ttot;
        if (WCSR && more) code_n = j < (ut_c.w & 511) ? (u32)codeC[ut_c.y + j] : 0u;
        PROF_MARK(0);
        if (ttot == 0) {  // uniform: every tile of the unit is empty
            if (more) issue(u + G, ut_c, ue_c, code_n);
            __syncthreads();
            continue;
        }
        if (WTILE && j < ns && tt > 0) {  // Ptr of the non-empty tile j (u16 x TM, vector stores)
            u16 pp[TM];
            int run = 0;
#pragma unroll
            for (int r = 0; r < TM; ++r) {
                pp[r] = (u16)run;
                run += __popc((w[r >> 1] >> ((r & 1) * 16)) & 0xffffu);
            }
            uint4 *dst = reinterpret_cast<uint4 *>(PtrC + (size_t)(t0 + j) * TM);
#pragma unroll
            for (int k = 0; k < TM / 8; ++k)
                dst[k] = make_uint4(pp[8 * k] | ((u32)pp[8 * k + 1] << 16), pp[8 * k + 2] | ((u32)pp[8 * k + 3] << 16),
                                    pp[8 * k + 4] | ((u32)pp[8 * k + 5] << 16),
                                    pp[8 * k + 6] | ((u32)pp[8 * k + 7] << 16));
        }
        const int nzbase = WTILE ? nnzoff[t0] : 0;
        __syncthreads();
        PROF_MARK(1);
        int s_lo = 0, s_hi = 0, base = 0, nz = 0;  // the current pass: tiles [s_lo, s_hi)
        // ---- W: outputs of a pass
        auto write_pass = [&]() {
            if (WCSR && !(ablate & 8)) {
                for (int eb = 0; eb < nz; eb += WG) {
                    const int e = eb + threadIdx.x;
                    const bool in = e < nz;
                    const int key = in ? (int)s_key[e] : 0;
                    const int r = in ? key >> 4 : TM;  // idle lanes match no row
                    int lrank = 0;
                    // rank among this wave's row-r nonzeros by four DPP wave scans of
                    // one-hot row counts (four rows x 8-bit fields per u32; a wave
                    // holds <= 64 of a row): no per-row ballot / exec-mask loop
                    {
                        const int g = r >> 2, sh = 8 * (r & 3);
                        u32 tot[4];
                        int pre = 0;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const u32 oh = (g == k) ? (1u << sh) : 0u;
                            const u32 inc = (u32)wave_incl_scan_dpp((int)oh);
                            tot[k] = (u32)__builtin_amdgcn_readlane((int)inc, 63);
                            pre = (g == k) ? (int)(((inc - oh) >> sh) & 0xffu) : pre;
                        }
                        lrank = pre;
                        if (lane < TM) {
                            const u32 t = (lane >> 2) == 0 ? tot[0] : (lane >> 2) == 1 ? tot[1]
                                        : (lane >> 2) == 2 ? tot[2] : tot[3];
                            s_wcnt[wv][lane] = (int)((t >> (8 * (lane & 3))) & 0xffu);
                        }
                    }
                    __syncthreads();
                    if (in) {
                        int before = s_run[r];
                        for (int w2 = 0; w2 < wv; ++w2) before += s_wcnt[w2][r];
                        const int dst = s_rowptr[r] + s_carry[r] + before + lrank;
                        csr_col[dst] = s_cols[s_kt[e]] * TM + (key & 15);
                        csr_val[dst] = acc[e];
                    }
                    __syncthreads();
                    if (threadIdx.x < TM) {
                        int add = 0;
                        for (int w2 = 0; w2 < WAVES; ++w2) add += s_wcnt[w2][threadIdx.x];
                        s_run[threadIdx.x] += add;
                    }
                    __syncthreads();  // s_wcnt is rewritten by the next 256 nonzeros
                }
            }
            if (WTILE) {
                if (j >= s_lo && j < s_hi && tt > 0) {
                    const int e0 = toff - base, out = nzbase + toff;
                    for (int k = 0; k < tt; ++k) {
                        ColC[out + k] = (u16)(s_key[e0 + k] & 15);
                        ValC[out + k] = acc[e0 + k];
                    }
                }
            }
            __syncthreads();
            if (WCSR && threadIdx.x < TM) s_carry[threadIdx.x] += s_run[threadIdx.x];
            __syncthreads();
            PROF_MARK(4);
        };
        for (;;) {
            int lo = s_lo + 1, hi = ns;  // largest s_hi with nnz(tiles s_lo..s_hi-1) <= NZCAP
            if (s_off[ns] - s_off[s_lo] <= S3_NZCAP) lo = ns;  // the rest fits one pass (the common case)
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_off[mid] - s_off[s_lo] <= S3_NZCAP) lo = mid; else hi = mid - 1;
            }
            s_hi = lo;
            base = s_off[s_lo];
            nz = s_off[s_hi] - base;
            if (nz == 0) break;  // uniform; only the last pass can be empty (it then runs to ns)
            // expand the pass's nonzeros (tile-major, then row-major in the tile)
            if (j >= s_lo && j < s_hi && tt > 0) {
                int e = toff - base;
                u32 wl[TW32];  // tile j's words, back from LDS
#pragma unroll
                for (int k = 0; k < NV4; ++k) {
                    const uint4 v = reinterpret_cast<const uint4 *>(s_mask + j * TW32)[k];
                    wl[4 * k] = v.x; wl[4 * k + 1] = v.y; wl[4 * k + 2] = v.z; wl[4 * k + 3] = v.w;
                }
#pragma unroll
                for (int r = 0; r < TM; ++r) {
                    u32 v = (wl[r >> 1] >> ((r & 1) * 16)) & 0xffffu;
                    while (v) {
                        const int hb = 31 - __clz(v);  // MSB-first: lowest column first
                        s_key[e] = (unsigned char)((r << 4) | (15 - hb));
                        s_kt[e++] = (unsigned char)j;
                        v &= ~(1u << hb);
                    }
                }
            }
            for (int e = threadIdx.x; e < nz; e += WG) acc[e] = 0.0;
            if (threadIdx.x < TM) s_run[threadIdx.x] = 0;
            __syncthreads();
            PROF_MARK(2);
            // ---- V: values
            if (!(ablate & 4)) {
                if (ELEM) {
                    const bool narrow = s_lo > 0 || s_hi < ns;
                    const int clo = s_cols[s_lo] * TM, chi = (s_cols[s_hi - 1] + 1) * TM;
                    elem_stream<TM>(E, ue, pre, s_rp, narrow, clo, chi, s_r, s_va, L, [&](int r, int slot, int pb) {
                        const int x = E.ciB[pb];
                        const double vb = E.vB[pb];
                        const int xt = (int)((u32)x / TM), c = (int)((u32)x % TM);  // x >= 0
                        const int sl = lower_bound_u(s_cols, s_lo, s_hi, xt);
                        if (sl >= s_hi || s_cols[sl] != xt) return;  // another pass's tile
                        const int rk = RST ? (int)s_rs[sl * TM + r] +
                                                 __popc(((s_mask[sl * TW32 + (r >> 1)] >> ((r & 1) * 16)) & 0xffffu) >>
                                                        (16 - c))
                                           : tile_rank16(s_mask + sl * TW32, r, c);
                        atomicAdd(&acc[s_off[sl] - base + rk], s_va[slot] * vb);
                    });
                } else {
                    const int a0 = V.Aptr[i], a1 = V.Aptr[i + 1];
                    for (int ab = a0; ab < a1; ab += WG) {
                        const int na = min(WG, a1 - ab);
                        const int tot = unit_setup(V, i, q, nu, a0, ab, na, L);
                        unit_items(V, ab, na, tot, s_cols, ns, L, [&](int a, int b, int sl) {
                            if (sl < s_lo || sl >= s_hi) return;
                            const int *br = V.rowsBrm + (size_t)b * (TN + 1);
                            const u32 *tile = s_mask + sl * TW32;
                            const int tb = s_off[sl] - base;
                            const int q1 = V.Annz[a + 1];
                            for (int qa = V.Annz[a]; qa < q1; ++qa) {
                                const int enc = V.ColA[qa];
                                const int r = enc / TN, c = enc - (enc / TN) * TN;
                                const int ks = br[c], ke = br[c + 1];
                                if (ks >= ke) continue;
                                const double va = V.ValA[qa];
                                for (int kb = ks; kb < ke; ++kb)
                                    atomicAdd(&acc[tb + tile_rank16(tile, r, V.ColB[kb])], va * V.ValB[kb]);
                            }
                        });
                        __syncthreads();
                    }
                }
            }
            PROF_MARK(3);
            if (s_hi == ns) break;  // the last pass writes after the next unit's loads are issued
            write_pass();
            s_lo = s_hi;
        }
        if (more) issue(u + G, ut_c, ue_c, code_n);  // in flight during the last pass's writes
        if (nz > 0) write_pass();
    }
}

// TSG_ABLATE (diagnostics bitmask, read once per process):
//    4  skip step 3's value pass        (results wrong)
//    8  skip step 3's CSR writes        (results wrong)
//   16  tile-payload value pass instead of element streaming (results correct)
//   64  per-phase clock totals, with the -DTSG_PROF_BUILD library (make prof)
//  256  step 1: no stored bitmasks       512  step 1: no unit-buffer emit (second product pass)
// 2048  tile counts: bitmap kernel only (no wave-per-tile-row count)
// 8192  CSR path: compact step 1's unit buffers into tile_columnidx (k_step1_gather)

// Step 1 (C tile structure = tile-pattern product of A's and B's row-major tile
// structures; includes tiles whose element product is empty, as the reference).
// Works for any tile sizes: only tile_ptr / tile_columnidx are read.  With CSR
// operands Ael/Bel (16x16): the element-level structure instead (non-empty C
// tiles only; the CSR path, whose C tiles are internal).
int dev_step1(Context &cx, const tsg_dev_tiles &A, const tsg_dev_tiles &B, tsg_dev_tiles &C,
              long long *tile_products_out, hipStream_t s, const tsg_dev_csr *Ael, const tsg_dev_csr *Bel,
              int2 *ebnd, long long **tbase_out, long long *tslots_out, bool fill_ebnd) {
    const bool el = Ael && Bel;  // element-level structure (16x16 tiles, CSR operands)
    if (el && !ebnd && Ael->nnz > 0) return TSG_ERR_INVALID;  // the element walks read the entry bounds
    const int tilemA = A.tilem, tilenB = B.tilen;
    int win, nwin;
    window_for(tilenB, &win, &nwin);
    if ((long)tilemA * nwin >= (1L << 31) - 1) return TSG_ERR_UNSUPPORTED;
    const long nunits1 = (long)tilemA * nwin;
    int *ucnt = nullptr;
    u64 *prod = nullptr;
    TSG_TRY(cx.get(&ucnt, (size_t)nunits1 + 1));
    TSG_TRY(cx.get(&prod, 1));
    TSG_TRY(cx.get(&C.tile_ptr, (size_t)tilemA + 1));
    const int g1 = grid_for(nunits1, 1, 16384);
    // k_step1_cap (element level) or k_step1_cap_tiles (tile level) runs, and zeroes these
    const bool capk = ((el && ebnd) || !el) && tilemA > 0 && !(ablate_bits() & 512);
    if (!capk) {
        TSG_HIP(hipMemsetAsync(prod, 0, sizeof(u64), s));
        TSG_HIP(hipMemsetAsync(ucnt + nunits1, 0, sizeof(int), s));
    }
    // keep each unit's bitmask (window/8 bytes) for the emit pass when that fits
    // 4 GiB: one tile-product enumeration instead of two
    // (and when the products per unit -- estimated from the mean B tile row --
    // outweigh a reread of the window's words, i.e. not for banded matrices)
    // EL with per-entry B bounds: pass 0 also emits each unit's sorted columns into
    // a unit buffer (capacity min(products, window)) when the buffers total at most
    // 2 x the element products + 2^26 slots; a gather compacts them after the scan
    int *ubuf = nullptr;
    long long *ubuf_off = nullptr;
    long long slots = 0;
    if (fill_ebnd && !capk) {  // no capacity kernel to fuse into
        k_entry_bounds<<<grid_for(Ael->nnz, WG, 16384), WG, 0, s>>>(Ael->columnindex, Ael->nnz, Bel->rowpointer,
                                                                   ebnd);
        fill_ebnd = false;
    }
    if (capk) {
        TSG_TRY(cx.get(&ubuf_off, (size_t)nunits1 + 1));
        if (el)
            k_step1_cap<<<grid_for((long)tilemA * 64, WG, 8192), WG, 0, s>>>(
                Ael->rowpointer, Ael->m, ebnd, tilemA, nwin, win, tilenB, ubuf_off,
                fill_ebnd ? Ael->columnindex : nullptr, fill_ebnd ? Bel->rowpointer : nullptr, prod, ucnt);
        else  // (the tile path's one walk: webbase's 62.5 K tile rows stored 512 MB of window bitmaps and read them back)
            k_step1_cap_tiles<<<grid_for((long)tilemA * 64, WG, 8192), WG, 0, s>>>(
                A.tile_ptr, A.tile_columnidx, B.tile_ptr, tilemA, nwin, win, tilenB, ubuf_off, prod, ucnt);
        fill_ebnd = false;
        TSG_HIP(hipGetLastError());
        TSG_TRY(scan_exclusive_i64(cx, ubuf_off, nunits1 + 1, s));
        TSG_TRY(read_i64(cx, ubuf_off + nunits1, &slots, s));
        const double est = el ? (double)Ael->nnz * ((double)Bel->nnz / (double)(Bel->m > 0 ? Bel->m : 1))
                              : (double)A.numtile * ((double)B.numtile / (double)(B.tilem > 0 ? B.tilem : 1));
        if ((double)slots <= 2.0 * est + (double)(1 << 26) && slots < (1LL << 31) &&
            cx.get(&ubuf, (size_t)slots + 1) == TSG_OK) {
        } else {
            (void)hipGetLastError();
            ubuf = nullptr;
            cx.put(ubuf_off);
            ubuf_off = nullptr;
        }
    }
    u32 *bmst = nullptr;
    const size_t bm_bytes = (size_t)nunits1 * (win / 8);
    const double est_products =
        el ? (double)Ael->nnz * ((double)Bel->nnz / (double)(Bel->m > 0 ? Bel->m : 1))
           : (double)A.numtile * ((double)B.numtile / (double)(B.tilem > 0 ? B.tilem : 1));
    const bool store = bm_bytes <= (4ull << 30) && est_products >= (double)nunits1 * (win / 32) / 8.0;
    if (store && !ubuf && !(ablate_bits() & 256) && cx.get(&bmst, bm_bytes / 4) != TSG_OK) {
        bmst = nullptr;
        (void)hipGetLastError();
    }
    if (tilemA > 0) {
        if (el)
            k_step1<0, true><<<g1, WG, 0, s>>>(Ael->rowpointer, Ael->columnindex, Bel->rowpointer, Bel->columnindex,
                                               tilemA, tilenB, nwin, win, ucnt, nullptr, nullptr, prod, bmst, Ael->m,
                                               ebnd, ubuf, ubuf_off);
        else
            k_step1<0><<<g1, WG, 0, s>>>(A.tile_ptr, A.tile_columnidx, B.tile_ptr, B.tile_columnidx, tilemA, tilenB,
                                         nwin, win, ucnt, nullptr, nullptr, prod, bmst, 0, nullptr, ubuf, ubuf_off);
    }
    TSG_HIP(hipGetLastError());
    long long numblk64 = 0, tile_products = 0;
    // one host round trip for the C tile count (overflow: > INT_MAX C tiles) and the product count
    TSG_TRY(scan_i32_total_impl(
        cx, ucnt, nunits1 + 1, s, &numblk64,
        [&] { k_rows_from_units<<<grid_for(tilemA + 1, WG, 4096), WG, 0, s>>>(ucnt, tilemA, nwin, C.tile_ptr); },
        reinterpret_cast<const long long *>(prod), &tile_products));
    const int numblkC = (int)numblk64;
    C.numtile = numblkC;
    const size_t nb1 = (size_t)numblkC + 1;
    if (tbase_out) *tbase_out = nullptr;
    // (only while the buffers are at most 2x the compacted tiles: step 2's mask
    // array is sized by the index space)
    if (ubuf && nwin == 1 && tbase_out && slots <= 2 * numblk64 + (1 << 20)) {
        // the caller indexes C tiles in unit-buffer space (tile row i's columns
        // start at ubuf_off[i]): no compaction; C.tile_columnidx is the buffer
        C.tile_columnidx = ubuf;
        *tbase_out = ubuf_off;
        *tslots_out = slots;
        cx.put(bmst);
        cx.put(ucnt);
        cx.put(prod);
        *tile_products_out = tile_products;
        return TSG_OK;
    }
    TSG_TRY(cx.get(&C.tile_columnidx, nb1));
    if (tilemA > 0) {
        if (ubuf)
            k_step1_gather<<<grid_for(nunits1, WAVES, 16384), WG, 0, s>>>(ubuf, ubuf_off, ucnt, nunits1,
                                                                           C.tile_columnidx);
        else if (bmst)
            k_step1<2><<<g1, WG, 0, s>>>(A.tile_ptr, A.tile_columnidx, B.tile_ptr, B.tile_columnidx, tilemA, tilenB,
                                         nwin, win, nullptr, ucnt, C.tile_columnidx, nullptr, bmst);
        else if (el)
            k_step1<1, true><<<g1, WG, 0, s>>>(Ael->rowpointer, Ael->columnindex, Bel->rowpointer, Bel->columnindex,
                                               tilemA, tilenB, nwin, win, nullptr, ucnt, C.tile_columnidx, nullptr,
                                               nullptr, Ael->m, ebnd);  // (the element walk reads ebnd)
        else
            k_step1<1><<<g1, WG, 0, s>>>(A.tile_ptr, A.tile_columnidx, B.tile_ptr, B.tile_columnidx, tilemA, tilenB,
                                         nwin, win, nullptr, ucnt, C.tile_columnidx, nullptr, nullptr);
    }
    TSG_HIP(hipGetLastError());
    cx.put(bmst);
    cx.put(ubuf);
    cx.put(ubuf_off);
    cx.put(ucnt);
    cx.put(prod);
    *tile_products_out = tile_products;
    return TSG_OK;
}

int dev_tilespgemm(Context &cx, const tsg_dev_tiles &A, const tsg_dev_tiles &B, tsg_dev_tiles &C,
                   tsg_stats *st, hipStream_t s, hipEvent_t *ev, tsg_dev_csr *csr_out, const tsg_dev_csr *Acsr,
                   const tsg_dev_csr *Bcsr, bool step2_elem) {
    ablate_bits();
    constexpr int TM = 16, TN = 16;
    if (A.tile_m != TM || A.tile_n != TN || B.tile_m != TN || B.tile_n != TM) return TSG_ERR_UNSUPPORTED;
    // element streaming needs the CSR operands (B rows column-sorted: caller's check)
    const bool have_csr = Acsr && Bcsr && Acsr->m == A.m && Bcsr->m == B.m;
    const bool s3elem = have_csr && !(g_ablate & 16);  // (tiled C out too: the host tile API with CSR)
    const bool s2elem = step2_elem && have_csr;
    const bool tilepay = !(s2elem && s3elem);  // some step reads the tile payloads
    if (A.n != B.m) return TSG_ERR_INVALID;
    if (!s2elem && (!B.rm_mask || !((A.tile_csr_Col && A.tile_nnz) || A.mask))) return TSG_ERR_INVALID;
    if (!s3elem && (!B.rm_rowstart || !A.tile_csr_Col || !A.tile_nnz)) return TSG_ERR_INVALID;
    const int tilemA = A.tilem, tilenB = B.tilen;
    C = tsg_dev_tiles{};
    C.m = A.m; C.n = B.n; C.tile_m = TM; C.tile_n = TM;
    C.tilem = tilemA; C.tilen = tilenB;
    if (ev) TSG_HIP(hipEventRecord(ev[0], s));
    // ---- step 1 ----
    // CSR path with element streaming: C's structure at element level (no empty tiles)
    const bool s1elem = csr_out && s2elem && s3elem;
    if (!s1elem && (!A.tile_columnidx || !B.tile_columnidx) && A.numtile > 0 && B.numtile > 0)
        return TSG_ERR_INVALID;  // tile-level step 1 needs both tile structures
    long long tile_products = 0;
    // per A entry: its B row's position range (step 1's element walk, the split points)
    int2 *ebnd = nullptr;
    if ((s2elem || s3elem) && Acsr->nnz > 0) {
        TSG_TRY(cx.get(&ebnd, (size_t)Acsr->nnz + 1));
        if (!s1elem) {  // (element step 1 fills them in its capacity kernel)
            k_entry_bounds<<<grid_for(Acsr->nnz, WG, 16384), WG, 0, s>>>(Acsr->columnindex, Acsr->nnz,
                                                                        Bcsr->rowpointer, ebnd);
            TSG_HIP(hipGetLastError());
        }
    }
    // CSR path: C tiles indexed in step 1's unit-buffer space when it allows (no
    // column compaction; C's tile arrays are internal there)
    long long *tbase = nullptr;
    long long tslots = 0;  // size of the C tile index space: numblkC, or the unit-buffer slots
    TSG_TRY(dev_step1(cx, A, B, C, &tile_products, s, s1elem ? Acsr : nullptr, s1elem ? Bcsr : nullptr,
                      s1elem ? ebnd : nullptr, (s1elem && !(g_ablate & 8192)) ? &tbase : nullptr, &tslots,
                      s1elem && ebnd));
    const int numblkC = C.numtile;
    const size_t nb1 = (size_t)numblkC + 1;
    if (!tbase) tslots = numblkC;
    if (ev) TSG_HIP(hipEventRecord(ev[1], s));
    // ---- step 2 ----
    int *uoff = nullptr, *urow = nullptr, *unit_rc = nullptr, *unit_rb = nullptr;
    int4 *utab = nullptr;
    const long maxu = (long)numblkC / CH + tilemA + 1;
    TSG_TRY(cx.get(&uoff, (size_t)tilemA + 1));
    TSG_TRY(cx.get(&urow, (size_t)maxu));
    TSG_TRY(cx.get(&utab, (size_t)maxu));
    TSG_TRY(cx.get(&unit_rc, (size_t)maxu * TM));
    if (!csr_out) TSG_TRY(cx.get(&C.tile_nnz, nb1));  // CSR path: row counts only, no tile nnz scan
    TSG_TRY(cx.get(&C.mask, ((size_t)tslots + 1) * CM<TM>::TW));
    // CSR path: step 2 hands step 3 a u16 code per C tile and full masks only for
    // tiles with > 1 nonzero (most webbase-like C tiles hold one nonzero)
    u16 *codeC = nullptr;
    if (csr_out) TSG_TRY(cx.get(&codeC, (size_t)tslots + 1));
    k_units_per_row<<<grid_for(tilemA, WG, 4096), WG, 0, s>>>(C.tile_ptr, tilemA, uoff);
    TSG_TRY(scan_exclusive_i32(cx, uoff, (long)tilemA + 1, s));
    k_unit_rows<<<grid_for(tilemA, WG, 4096), WG, 0, s>>>(uoff, C.tile_ptr, tilemA, urow, utab, tbase);
    if (C.tile_nnz) k_set_i32<<<1, 1, 0, s>>>(C.tile_nnz + numblkC, 0);
    TSG_HIP(hipGetLastError());
    // element split tables: sizes queued ahead of the unit count's read (one round trip)
    long long *ebase = nullptr;
    if (s2elem || s3elem) {
        TSG_TRY(cx.get(&ebase, (size_t)tilemA + 1));
        k_esplit_counts<TM><<<grid_for(tilemA, WG, 4096), WG, 0, s>>>(uoff, Acsr->rowpointer, A.m, tilemA, ebase);
        TSG_TRY(scan_exclusive_i64(cx, ebase, (long)tilemA + 1, s));
    }
    int nunits = 0;
    long long ne = 0;
    TSG_HIP(hipMemcpyAsync(cx.pinned, uoff + tilemA, sizeof(int), hipMemcpyDeviceToHost, s));
    if (ebase) TSG_HIP(hipMemcpyAsync(cx.pinned64, ebase + tilemA, sizeof(long long), hipMemcpyDeviceToHost, s));
    TSG_TRY(stream_wait(s));
    nunits = cx.pinned[0];
    if (ebase) ne = cx.pinned64[0];
    const int gu = grid_for(maxu, 1, TSG_GU_CAP);  // workgroups of steps 2 and 3 (units strided over them)
    // tile-product split points: every A tile's B tile row cut at its C tile row's unit boundaries
    long long *sbase = nullptr;
    int *split = nullptr;
    if (tilepay) {
        TSG_TRY(cx.get(&sbase, (size_t)tilemA + 1));
        k_split_counts<<<grid_for(tilemA, WG, 4096), WG, 0, s>>>(uoff, A.tile_ptr, tilemA, sbase);
        TSG_TRY(scan_exclusive_i64(cx, sbase, (long)tilemA + 1, s));
        long long nsplit = 0;
        TSG_TRY(read_i64(cx, sbase + tilemA, &nsplit, s));
        TSG_TRY(cx.get(&split, (size_t)nsplit + 1));
        int *trowA = A.tile_rowidx;
        if (!trowA) {
            TSG_TRY(cx.get(&trowA, (size_t)A.numtile + 1));
            k_crow<<<grid_for(tilemA, WAVES, 8192), WG, 0, s>>>(A.tile_ptr, tilemA, trowA);
        }
        if (A.numtile > 0)
            k_unit_splits<<<grid_for(A.numtile, WG, 8192), WG, 0, s>>>(A.numtile, trowA, A.tile_ptr,
                                                                      A.tile_columnidx, B.tile_ptr, B.tile_columnidx,
                                                                      uoff, C.tile_ptr, C.tile_columnidx, sbase, split);
        TSG_HIP(hipGetLastError());
        if (trowA != A.tile_rowidx) cx.put(trowA);
    }
    const ABView V{A.tile_ptr, A.tile_columnidx, A.tile_nnz, A.tile_csr_Col, A.tile_csr_Value,
                   B.tile_ptr, B.tile_columnidx, B.rm_mask, B.rm_rowstart, B.tile_csr_Col, B.tile_csr_Value,
                   split, sbase, A.mask};
    // element split points: every A entry's B CSR row cut at the unit boundaries (+ row end)
    ECsr E{};
    int *esplit = nullptr;
    int4 *etab = nullptr;
    if (s2elem || s3elem) {
        TSG_TRY(cx.get(&esplit, (size_t)ne + 1));
        E = ECsr{A.m, Acsr->rowpointer, Acsr->columnindex, Acsr->value, Bcsr->rowpointer, Bcsr->columnindex,
                 Bcsr->value, esplit, ebase};
        TSG_TRY(cx.get(&etab, (size_t)maxu));
        if (nunits > 0) {
            k_unit_etab<TM><<<grid_for(nunits, WG, 8192), WG, 0, s>>>(utab, nunits, Acsr->rowpointer, A.m, ebase,
                                                                      etab);
            k_esplit_units<TM><<<grid_for(nunits, WAVES, 16384), WG, 0, s>>>(utab, etab, nunits, ebnd,
                                                                             Bcsr->columnindex, C.tile_columnidx,
                                                                             esplit);
        }
        TSG_HIP(hipGetLastError());
    }
    if (g_ablate & 64) {
        unsigned long long z[16] = {};
        TSG_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_prof), z, sizeof(z), 0, hipMemcpyHostToDevice, s));
    }
    if (numblkC > 0) {
        if (s2elem)
            k_step2<TM, TN, true><<<gu, WG, 0, s>>>(utab, etab, nunits, V, E, C.tile_columnidx, C.tile_nnz, unit_rc,
                                                    C.mask, codeC, g_ablate);
        else
            k_step2<TM, TN, false><<<gu, WG, 0, s>>>(utab, etab, nunits, V, E, C.tile_columnidx, C.tile_nnz, unit_rc,
                                                     C.mask, codeC, g_ablate);
    }
    TSG_HIP(hipGetLastError());
    long long nnz64 = 0;
    // element path: nnz(C) is bounded by the element products (known on the host
    // since step 1), so its read-back waits for the end of the pipeline
    const bool defer_nnz = csr_out && s1elem && tile_products <= 0x7ffffffell && !(g_ablate & 16384);
    if (!csr_out) TSG_TRY(scan_exclusive_i32_total(cx, C.tile_nnz, (long)numblkC + 1, s, &nnz64));  // fits int32
    if (csr_out) {
        csr_out->m = A.m;
        csr_out->n = B.n;
        TSG_TRY(cx.get(&csr_out->rowpointer, (size_t)A.m + 1));
        TSG_TRY(cx.get(&unit_rb, (size_t)maxu * TM));
        k_set_i32<<<1, 1, 0, s>>>(csr_out->rowpointer + A.m, 0);
        if (tilemA > 0)
            k_unit_rowbase<TM><<<grid_for((long)tilemA * TM, WG, 8192), WG, 0, s>>>(uoff, tilemA, A.m, unit_rc, unit_rb,
                                                                                  csr_out->rowpointer);
        TSG_HIP(hipGetLastError());
        if (defer_nnz)  // nnz(C) <= element products <= INT_MAX: read back after step 3
            TSG_TRY(scan_exclusive_i32(cx, csr_out->rowpointer, (long)A.m + 1, s));
        else
            TSG_TRY(scan_exclusive_i32_total(cx, csr_out->rowpointer, (long)A.m + 1, s, &nnz64));  // fits int32
    }
    // (deferred: the element-product bound sizes step 3's outputs)
    int nnzC = defer_nnz ? (int)tile_products : (int)nnz64;
    C.nnz = nnzC;
    if (ev) TSG_HIP(hipEventRecord(ev[2], s));
    // ---- step 3 ----
    if (csr_out) {
        csr_out->nnz = nnzC;
        TSG_TRY(cx.get(&csr_out->columnindex, (size_t)nnzC + 1));
        TSG_TRY(cx.get(&csr_out->value, (size_t)nnzC + 1));
    } else {
        TSG_TRY(cx.get(&C.tile_csr_Ptr, nb1 * TM));
        TSG_TRY(cx.get(&C.tile_csr_Col, (size_t)nnzC + 1));
        TSG_TRY(cx.get(&C.tile_csr_Value, (size_t)nnzC + 1));
    }
    if (ev) TSG_HIP(hipEventRecord(ev[4], s));
    if (csr_out) {
        if (nnzC > 0 || defer_nnz) {
            if (s3elem && !s2elem)  // denser tiles: row-start table
                k_step3<TM, TN, true, false, true, true><<<gu, WG, 0, s>>>(
                    utab, etab, nunits, A.m, V, E, C.tile_columnidx, C.tile_nnz, C.mask, codeC, unit_rb,
                    csr_out->rowpointer, csr_out->columnindex, csr_out->value, nullptr, nullptr, nullptr, g_ablate);
            else if (s3elem)
                k_step3<TM, TN, true, false, true><<<gu, WG, 0, s>>>(
                    utab, etab, nunits, A.m, V, E, C.tile_columnidx, C.tile_nnz, C.mask, codeC, unit_rb,
                    csr_out->rowpointer, csr_out->columnindex, csr_out->value, nullptr, nullptr, nullptr, g_ablate);
            else
                k_step3<TM, TN, true, false, false><<<gu, WG, 0, s>>>(
                    utab, etab, nunits, A.m, V, E, C.tile_columnidx, C.tile_nnz, C.mask, codeC, unit_rb,
                    csr_out->rowpointer, csr_out->columnindex, csr_out->value, nullptr, nullptr, nullptr, g_ablate);
        }
    } else if (nnzC > 0) {  // the reference's tiled C (Ptr, Col, Value per tile)
        if (s3elem && !s2elem)
            k_step3<TM, TN, false, true, true, true><<<gu, WG, 0, s>>>(
                utab, etab, nunits, A.m, V, E, C.tile_columnidx, C.tile_nnz, C.mask, nullptr, nullptr, nullptr,
                nullptr, nullptr, C.tile_csr_Ptr, C.tile_csr_Col, C.tile_csr_Value, g_ablate);
        else if (s3elem)
            k_step3<TM, TN, false, true, true><<<gu, WG, 0, s>>>(
                utab, etab, nunits, A.m, V, E, C.tile_columnidx, C.tile_nnz, C.mask, nullptr, nullptr, nullptr,
                nullptr, nullptr, C.tile_csr_Ptr, C.tile_csr_Col, C.tile_csr_Value, g_ablate);
        else
            k_step3<TM, TN, false, true, false><<<gu, WG, 0, s>>>(
                utab, etab, nunits, A.m, V, E, C.tile_columnidx, C.tile_nnz, C.mask, nullptr, nullptr, nullptr,
                nullptr, nullptr, C.tile_csr_Ptr, C.tile_csr_Col, C.tile_csr_Value, g_ablate);
    }
    TSG_HIP(hipGetLastError());
    if (ev) TSG_HIP(hipEventRecord(ev[5], s));
    if (g_ablate & 64) {
        unsigned long long pr[16];
        TSG_HIP(hipMemcpyFromSymbolAsync(pr, HIP_SYMBOL(g_prof), sizeof(pr), 0, hipMemcpyDeviceToHost, s));
        TSG_TRY(stream_wait(s));
        double tot = 0, tot2 = 0;
        for (int k = 0; k < 8; ++k) tot += (double)pr[k];
        for (int k = 8; k < 16; ++k) tot2 += (double)pr[k];
        fprintf(stderr, "k_step2 phases (%% of WG-0 clock): load %.1f stream %.1f tail %.1f  total %.3g\n",
                100 * pr[8] / tot2, 100 * pr[9] / tot2, 100 * pr[10] / tot2, tot2);
        fprintf(stderr, "k_step3 phases (%% of WG-0 clock): load %.1f prologue %.1f passinit %.1f values %.1f "
                "write %.1f gap %.1f  total %.3g\n", 100 * pr[0] / tot, 100 * pr[1] / tot, 100 * pr[2] / tot,
                100 * pr[3] / tot, 100 * pr[4] / tot, 100 * pr[7] / tot, tot);
    }
    cx.put(tbase);
    cx.put(esplit);
    cx.put(ebase);
    cx.put(etab);
    cx.put(codeC);
    cx.put(ebnd);
    cx.put(uoff);
    cx.put(urow);
    cx.put(utab);
    cx.put(unit_rc);
    cx.put(unit_rb);
    cx.put(split);
    cx.put(sbase);
    if (ev) TSG_HIP(hipEventRecord(ev[3], s));
    if (defer_nnz) {  // the pipeline's one read-back after step 3
        TSG_HIP(hipMemcpyAsync(cx.pinned, csr_out->rowpointer + A.m, sizeof(int), hipMemcpyDeviceToHost, s));
        TSG_TRY(stream_wait(s));
        nnzC = cx.pinned[0];
        C.nnz = nnzC;
        csr_out->nnz = nnzC;
    }
    if (st) {
        st->numblkC = numblkC;
        st->nnzC = nnzC;
        st->tile_products = tile_products;
    }
    return TSG_OK;
}

// Ptr and mask of structurally empty C tiles := 0: a thread per tile, its
// tm u16 of Ptr (tm*tm/16 of mask) written as 16-byte vectors
__global__ __launch_bounds__(WG) void k_zero_empty_ptr(const int *nnzoff, int numtile, int tm, u16 *Ptr, u16 *mask) {
    const int pv = tm / 8, mv = tm * (tm / 16) / 8;  // uint4 per tile
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    for (long t = (long)blockIdx.x * WG + threadIdx.x; t < numtile; t += (long)gridDim.x * WG) {
        if (nnzoff[t + 1] != nnzoff[t]) continue;
        uint4 *p = reinterpret_cast<uint4 *>(Ptr + t * tm);
        for (int k = 0; k < pv; ++k) p[k] = z;
        if (mask) {
            uint4 *q = reinterpret_cast<uint4 *>(mask + t * tm * (tm / 16));
            for (int k = 0; k < mv; ++k) q[k] = z;
        }
    }
}

// Reference-layout extras for the host drop-in API: zero Ptr of empty C tiles
// and fill tile_rowidx (the device pipeline needs neither).
int dev_tiles_finalize_c(Context &cx, tsg_dev_tiles &C, hipStream_t s, bool zero_empty) {
    if (C.numtile <= 0) return TSG_OK;
    if (zero_empty)
        k_zero_empty_ptr<<<grid_for(C.numtile, WG, 16384), WG, 0, s>>>(C.tile_nnz, C.numtile, C.tile_m, C.tile_csr_Ptr,
                                                                  C.mask);
    TSG_TRY(cx.get(&C.tile_rowidx, (size_t)C.numtile + 1));
    k_crow<<<grid_for(C.tilem, WAVES, 8192), WG, 0, s>>>(C.tile_ptr, C.tilem, C.tile_rowidx);
    TSG_HIP(hipGetLastError());
    return TSG_OK;
}

// rm2csc for a B tiling that arrives from the host (row-major + CSC structure):
// CSC position p of tile (ti, j) -> its index in the row-major structure.
__global__ __launch_bounds__(WG) void k_rm2csc(const int *tile_ptr, const int *tcol, const int *csc_ptr,
                                               const int *csc_rowidx, int tilen, int numtile, int *rm2csc) {
    for (int p = blockIdx.x * WG + threadIdx.x; p < numtile; p += gridDim.x * WG) {
        int lo = 0, hi = tilen;  // last j with csc_ptr[j] <= p
        while (lo < hi) {
            int mid = (lo + hi + 1) >> 1;
            if (csc_ptr[mid] <= p) lo = mid; else hi = mid - 1;
        }
        const int j = lo, ti = csc_rowidx[p];
        const int rm = lower_bound_dev(tcol, tile_ptr[ti], tile_ptr[ti + 1], j);
        rm2csc[rm] = p;
    }
}

// B's row-major views, one thread per output element (coalesced stores):
// rm_rowstart[t][c] = absolute start of row c of row-major tile t (c = tn: its
// end), rm_mask[t][k] = its mask word k
__global__ __launch_bounds__(WG) void k_build_b_aux(int numtile, int tn, int mw, const int *rm2csc, const int *Bnnz,
                                                     const u16 *PtrB, const u16 *maskB, u16 *rm_mask, int *rm_rowstart) {
    const long nrs = (long)numtile * (tn + 1), nmk = (long)numtile * tn * mw;
    for (long x = (long)blockIdx.x * WG + threadIdx.x; x < nrs + nmk; x += (long)gridDim.x * WG) {
        if (x < nrs) {
            const int t = (int)(x / (tn + 1)), c = (int)(x - (long)t * (tn + 1));
            const int bc = rm2csc[t];
            rm_rowstart[x] = c < tn ? Bnnz[bc] + PtrB[(size_t)bc * tn + c] : Bnnz[bc + 1];
        } else {
            const long y = x - nrs;
            const int t = (int)(y / (tn * mw)), k = (int)(y - (long)t * tn * mw);
            rm_mask[y] = maskB[(size_t)rm2csc[t] * tn * mw + k];
        }
    }
}

int dev_rm2csc_from_structs(Context &cx, tsg_dev_tiles &B, hipStream_t s) {
    TSG_TRY(cx.get(&B.tile_rm2csc, (size_t)B.numtile + 1));
    if (B.numtile > 0)
        k_rm2csc<<<grid_for(B.numtile, WG, 8192), WG, 0, s>>>(B.tile_ptr, B.tile_columnidx, B.csc_tile_ptr,
                                                             B.csc_tile_rowidx, B.tilen, B.numtile, B.tile_rm2csc);
    TSG_TRY(cx.get(&B.rm_mask, ((size_t)B.numtile + 1) * B.tile_m * (B.tile_n / 16)));
    TSG_TRY(cx.get(&B.rm_rowstart, ((size_t)B.numtile + 1) * (B.tile_m + 1)));
    if (B.numtile > 0)
        k_build_b_aux<<<grid_for((long)B.numtile * (2 * B.tile_m + 1), WG, 16384), WG, 0, s>>>(B.numtile, B.tile_m, B.tile_n / 16, B.tile_rm2csc,
                                                                  B.tile_nnz, B.tile_csr_Ptr, B.mask, B.rm_mask,
                                                                  B.rm_rowstart);
    TSG_HIP(hipGetLastError());
    return TSG_OK;
}

// ---------------------------------------------------------------------------
// tile2csr (tile2csr.h:72-140).  Wave per C tile row; lane = tile.  Pass 1 sums
// per-row counts; pass 2 carries 16 running row offsets across 64-tile chunks.
// ---------------------------------------------------------------------------
template <int TM>
__global__ __launch_bounds__(WG) void k_t2c_count(const int *Cptr, int tilem, int m, const int *nnzoff,
                                                  const u16 *Ptr, int *rowcnt) {
    const int lane = lane_id();
    const int gw = (blockIdx.x * WG + threadIdx.x) >> 6, nw = gridDim.x * WAVES;
    for (int i = gw; i < tilem; i += nw) {
        int cnt[TM];
#pragma unroll
        for (int r = 0; r < TM; ++r) cnt[r] = 0;
        for (int base = Cptr[i]; base < Cptr[i + 1]; base += 64) {
            const int t = base + lane;
            if (t < Cptr[i + 1]) {
                const int o0 = nnzoff[t], tnz = nnzoff[t + 1] - o0;
                if (tnz) {
                    const u16 *p = Ptr + (size_t)t * TM;
#pragma unroll
                    for (int r = 0; r < TM; ++r) {
                        int nx = (r == TM - 1) ? tnz : (int)p[r + 1];
                        cnt[r] += nx - (int)p[r];
                    }
                }
            }
        }
#pragma unroll
        for (int r = 0; r < TM; ++r) {
            int v = wave_sum(cnt[r]);
            if (lane == r && i * TM + r < m) rowcnt[i * TM + r] = v;
        }
    }
}

template <int TM>
__global__ __launch_bounds__(WG) void k_t2c_fill(const int *Cptr, const int *Ccol, int tilem, int m,
                                                 const int *nnzoff, const u16 *Ptr, const u16 *ColC,
                                                 const double *ValC, const int *rowptr, int *col, double *val) {
    const int lane = lane_id();
    const int gw = (blockIdx.x * WG + threadIdx.x) >> 6, nw = gridDim.x * WAVES;
    for (int i = gw; i < tilem; i += nw) {
        const int rowlen = min(TM, m - i * TM);
        int carry[TM];
#pragma unroll
        for (int r = 0; r < TM; ++r) carry[r] = 0;
        for (int base = Cptr[i]; base < Cptr[i + 1]; base += 64) {
            const int t = base + lane;
            const bool in = t < Cptr[i + 1];
            int o0 = 0, tnz = 0;
            if (in) { o0 = nnzoff[t]; tnz = nnzoff[t + 1] - o0; }
            if (__ballot(tnz > 0) == 0ull) continue;
            const u16 *p = Ptr + (size_t)(in ? t : 0) * TM;
            const int tc = in ? Ccol[t] : 0;
#pragma unroll
            for (int r = 0; r < TM; ++r) {
                int st = tnz ? (int)p[r] : 0;
                int nx = tnz ? ((r == TM - 1) ? tnz : (int)p[r + 1]) : 0;
                int c = nx - st;
                int inc = wave_incl_scan(c);
                int dst0 = carry[r] + inc - c;
                carry[r] += wave_last(inc);
                if (r < rowlen && c > 0) {
                    const int R = i * TM + r;
                    int d = rowptr[R] + dst0;
                    for (int k = 0; k < c; ++k) {
                        col[d + k] = tc * TM + (int)ColC[o0 + st + k];
                        val[d + k] = ValC[o0 + st + k];
                    }
                }
            }
        }
    }
}

template <int TM>
static void t2c_launch_count(const tsg_dev_tiles &C, int *rowcnt, int g, hipStream_t s) {
    k_t2c_count<TM><<<g, WG, 0, s>>>(C.tile_ptr, C.tilem, C.m, C.tile_nnz, C.tile_csr_Ptr, rowcnt);
}

template <int TM>
static void t2c_launch_fill(const tsg_dev_tiles &C, tsg_dev_csr &out, int g, hipStream_t s) {
    k_t2c_fill<TM><<<g, WG, 0, s>>>(C.tile_ptr, C.tile_columnidx, C.tilem, C.m, C.tile_nnz, C.tile_csr_Ptr,
                                    C.tile_csr_Col, C.tile_csr_Value, out.rowpointer, out.columnindex, out.value);
}

int dev_tile2csr(Context &cx, const tsg_dev_tiles &C, tsg_dev_csr &out, hipStream_t s) {
    if (!tile_side_supported(C.tile_m)) return TSG_ERR_UNSUPPORTED;
    out.m = C.m;
    out.n = C.n;
    out.nnz = C.nnz;
    TSG_TRY(cx.get(&out.rowpointer, (size_t)C.m + 1));
    TSG_TRY(cx.get(&out.columnindex, (size_t)C.nnz + 1));
    TSG_TRY(cx.get(&out.value, (size_t)C.nnz + 1));
    TSG_HIP(hipMemsetAsync(out.rowpointer, 0, ((size_t)C.m + 1) * sizeof(int), s));
    const int g = grid_for(C.tilem, WAVES, 8192);
    if (C.tilem > 0) {
        if (C.tile_m == 16) t2c_launch_count<16>(C, out.rowpointer, g, s);
        else if (C.tile_m == 32) t2c_launch_count<32>(C, out.rowpointer, g, s);
        else if (C.tile_m == 48) t2c_launch_count<48>(C, out.rowpointer, g, s);
        else t2c_launch_count<64>(C, out.rowpointer, g, s);
    }
    TSG_HIP(hipGetLastError());
    TSG_TRY(scan_exclusive_i32(cx, out.rowpointer, (long)C.m + 1, s));
    if (C.tilem > 0 && C.nnz > 0) {
        if (C.tile_m == 16) t2c_launch_fill<16>(C, out, g, s);
        else if (C.tile_m == 32) t2c_launch_fill<32>(C, out, g, s);
        else if (C.tile_m == 48) t2c_launch_fill<48>(C, out, g, s);
        else t2c_launch_fill<64>(C, out, g, s);
    }
    TSG_HIP(hipGetLastError());
    return TSG_OK;
}

}  // namespace tsg
