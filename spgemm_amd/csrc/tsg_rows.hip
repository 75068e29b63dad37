// tsg_rows.hip -- row-merge path of the element TileSpGEMM for gfx950 (wave64):
// C = A*B, device CSR in -> device CSR out, B's rows column-sorted, for
// operands whose C rows are long and spread over the whole column range with
// little merging (web graphs such as webbase-1M: 69 M element products give
// 65 M nonzeros, so C is nearly the product expansion itself).
//
// Reference semantics (paths under /root/reference/src): the same C as steps
// 1-3 + tile2csr (tilespgemm-cuda.h:279-2218, tile2csr.h:72-140) -- every C
// row the column-sorted union of the scaled B rows its A entries select, equal
// columns summed.  The reference reaches it through the tile structure; here a
// row's B rows ARE its sorted runs, so the row is built by merging them:
//
//   * entry table: each A entry's B range and a prefix of the element products
//     over all entries (one int64 scan) -- a row's products, its staging
//     offset and its runs' offsets are differences of that prefix;
//   * rows binned by products (and runs) into four classes, each with a kernel
//     shaped for it:
//       S  <= 64 products : a wave per row, ranks by counting in registers;
//       M1 <= 512         : a wave per row, pairwise merges of the runs in LDS;
//       M2 <= 4,096       : a workgroup per row, the same merges;
//       H  longer         : a workgroup per row, a bitmap of a column window in
//                           LDS, ranks by popcount, values by f64 atomics;
//     the merge keys are (column, run, position) so they are unique and the
//     merged order -- hence every sum's order -- is deterministic (class H's
//     atomics are the exception);
//   * each row writes its nonzeros, column-sorted, to a staging area at the
//     prefix of the products (products bound nnz), and its nnz; a scan of the
//     counts gives the CSR row pointers, one streaming pass the final arrays.
#include "tsg_internal.h"
#include "tsg_dev_common.h"

#include <cstdio>
#include <cstdlib>

namespace tsg {

namespace {

constexpr int S16_MAX = 16;           // class S16: products (and runs) per row, 4 rows per wave
constexpr int RS_MAX = 64;            // class S64: products (and runs) per row, a wave
constexpr int CP_CH = 2048;           // positions per chunk of the compaction (k_rows_compact)
constexpr int S16_U = 2, S64_U = 2;   // rows per lane group of the S16 / S64 kernels (k_rows_small; S16 at
                                      // U = 4: 95 vs 86 us on mc2depi; U = 2: 4 us under U = 1)
// merge classes M1..M4: products and runs per row, threads per row -- each
// sized so its LDS (16 B per product + 16 B per run) keeps several rows per CU
// (M0..M3: run tables a few runs short of a power of two, so that 32, 16, 8
// and 4 workgroups fit a CU's 160 KiB of LDS -- full 64/128/256/512-run tables
// made each workgroup a few dozen bytes too large for the last one)
constexpr int M0_CAP = 256, M0_RUNS = 62, M0_NT = 64;      // 5,104 B: one wave per row
constexpr int M1_CAP = 512, M1_RUNS = 124, M1_NT = 128;    // 10,208 B
constexpr int M2_CAP = 1024, M2_RUNS = 248, M2_NT = 256;   // 20,400 B
constexpr int M3_CAP = 2048, M3_RUNS = 504, M3_NT = 512;   // 40,912 B
constexpr int M4_CAP = 4096, M4_RUNS = 512, M4_NT = 1024;  // 72 KB
constexpr int W_CH = 32768;           // windowed rows: products per chunk (k_rows_wcount / wscatter)
constexpr int NCLS = 8;               // S16, S64, M0..M4, H
constexpr int DR_SMAX = 4096;         // hub rows: products outside the dominant run (the DR kernels)
constexpr int DR_CH = 16384;          // DR fill: dominant-run elements per chunk
constexpr int DR_GR = 16;             // DR fill: rows of one run per chunk (the run's range read once for them)
constexpr int DR_GMAX = 8192;         // DR rows grouped by run in one workgroup's LDS (more: a chunk per row)
constexpr int BIN_ROWS = 2048;        // rows per workgroup of the binning kernel
constexpr int RH_NT = 1024;           // class H: workgroup
constexpr int RH_WORDS = 16384;       // class H: bitmap words (u64) per window: 128 KB of LDS
constexpr long long RH_SPAN = (long long)RH_WORDS * 64;  // columns per window (1,048,576)
constexpr int RH_BLK = 512;           // words per rank block (int prefix); u16 prefix per 4-word group inside
constexpr int RH_NBLK = RH_WORDS / RH_BLK;
constexpr int RH_NGRP = RH_WORDS / 4;
constexpr int RH_PPT = 16;            // class H, one-walk rows: products per thread held in registers
constexpr int OW_CH = RH_PPT * RH_NT;  // ... so many per row (past it: the row's scratch slots)
constexpr int OW_CV = 2 * RH_WORDS;    // column ranks per pass (int in the bitmap's LDS)
constexpr int OW_RUNS = 2 * RH_NT;     // runs of a one-walk row (two per thread)
static_assert(OW_CH <= RH_WORDS, "one-walk rows: a pass's values fit the bitmap's LDS");

__device__ __forceinline__ u32 lanes_below(u64 b) {
    return __builtin_amdgcn_mbcnt_hi((u32)(b >> 32), __builtin_amdgcn_mbcnt_lo((u32)b, 0u));
}
__device__ __forceinline__ int key_col(u64 k) { return (int)(k >> 32); }

}  // namespace

// TSG_ROWS_PROF builds (make prof): per-phase wall-clock totals of the class
// kernels' workgroups (thread 0 after each phase's barrier), printed per call
#ifdef TSG_ROWS_PROF
__device__ unsigned long long g_rows_prof[3][256][12];  // (spread over 256 slots: few same-address atomics)
#define RP_INIT unsigned long long rp_acc[12] = {}, rp_t = wall_clock64();
#define RP(k)                                         \
    do {                                              \
        const unsigned long long _t = wall_clock64(); \
        rp_acc[k] += _t - rp_t;                       \
        rp_t = _t;                                    \
    } while (0)
#define RP_DONE(K)                                                          \
    do {                                                                    \
        if (threadIdx.x == 0)                                               \
            for (int _k = 0; _k < 12; ++_k) atomicAdd(&g_rows_prof[K][blockIdx.x & 255][_k], rp_acc[_k]); \
    } while (0)
#else
#define RP_INIT
#define RP(k) \
    do {      \
    } while (0)
#define RP_DONE(K) \
    do {           \
    } while (0)
#endif

struct RowsArgs {
    const int *rpA;
    const double *vA;
    const int2 *ebnd;      // per A entry: its B row's [start, end)
    const long long *E;    // per A entry: prefix of the element products (E[nnzA] = all)
    const int *Bcol;
    const double *Bval;
    const int4 *list;      // the class's rows: (row, first A entry, A entries, -)
    int nrows;
    int *rnnz;             // nnz of each row (the row pointers after a scan)
    int *Scol;             // staging: row r's nonzeros from E[rpA[r]]
    double *Sval;
};

// per A entry: its B row's range and products (the latter scanned into E)
// (also zeroes the binning kernel's counters: no separate memset in the stream)
__global__ __launch_bounds__(WG) void k_rows_entries(const int *ciA, long nnzA, const int *rpB, int2 *ebnd,
                                                     long long *E, int *cls) {
    if (blockIdx.x == 0 && threadIdx.x < 32) cls[threadIdx.x] = 0;  // (class counts, statistics, cursors)
    for (long a = (long)blockIdx.x * WG + threadIdx.x; a <= nnzA; a += (long)gridDim.x * WG) {
        if (a == nnzA) {
            E[a] = 0;
            break;
        }
        const int k = ciA[a], b0 = rpB[k], b1 = rpB[k + 1];
        ebnd[a] = make_int2(b0, b1);
        E[a] = b1 - b0;
    }
}

// ---- the setup's and the row pointers' scans fused with their neighbours: at
// mc2depi's size every launch costs 4-5 us however little it does, and the
// generic scan is three (block sums, their scan, apply).  Up to RS_INLINE_MAX
// tiles, each apply workgroup adds up the earlier tiles' sums itself.
constexpr int RS_ITEMS = 16, RS_TILE = WG * RS_ITEMS;
constexpr int RS_INLINE_MAX = 2048;
__device__ __forceinline__ int rs_pad(int i) { return i + (i >> 4); }

// the entry table with the first half of its scan: per A entry its B row's
// range and products, per tile of RS_TILE entries their sum (E[nnzA] = 0: the
// n+1 slot); also zeroes the binning kernel's counters
__global__ __launch_bounds__(WG) void k_rows_entries_sum(const int *ciA, long nnzA, const int *rpB, int2 *ebnd,
                                                         long long *E, int *cls, long long *part) {
    __shared__ long long red[WAVES];
    const int tid = threadIdx.x;
    if (blockIdx.x == 0 && tid < 32) cls[tid] = 0;  // (class counts, statistics, cursors)
    const long base = (long)blockIdx.x * RS_TILE;
    int kk[RS_ITEMS];
#pragma unroll
    for (int u = 0; u < RS_ITEMS; ++u) {
        const long a = base + u * WG + tid;
        kk[u] = a < nnzA ? ciA[a] : 0;
    }
    int b0[RS_ITEMS], b1[RS_ITEMS];
#pragma unroll
    for (int u = 0; u < RS_ITEMS; ++u) {
        const long a = base + u * WG + tid;
        b0[u] = a < nnzA ? rpB[kk[u]] : 0;
        b1[u] = a < nnzA ? rpB[kk[u] + 1] : 0;
    }
    long long sum = 0;
#pragma unroll
    for (int u = 0; u < RS_ITEMS; ++u) {
        const long a = base + u * WG + tid;
        if (a < nnzA) {
            ebnd[a] = make_int2(b0[u], b1[u]);
            E[a] = b1[u] - b0[u];
            sum += b1[u] - b0[u];
        } else if (a == nnzA) {
            E[a] = 0;
        }
    }
    sum = block_sum(sum, red);
    if (tid == 0) part[blockIdx.x] = sum;
}

// per tile of RS_TILE values their sum
template <class T>
__global__ __launch_bounds__(WG) void k_rows_count_sum(const T *a, long n, T *part) {
    __shared__ T red[WAVES];
    const long base = (long)blockIdx.x * RS_TILE;
    T sum = 0;
#pragma unroll
    for (int u = 0; u < RS_ITEMS; ++u) {
        const long i = base + u * WG + threadIdx.x;
        sum += i < n ? a[i] : 0;
    }
    sum = block_sum(sum, red);
    if (threadIdx.x == 0) part[blockIdx.x] = sum;
}

// the exclusive scan's apply, the tile's prefix summed from the earlier tiles'
// sums.  CFIRST (the row pointers, n = m + 1): also the compaction's chunk
// table (k_rows_cfirst's job: the row holding each chunk's first position) and
// nnz(C) (the scan's last value) into the caller's host-mapped *hnnz.
template <class T, bool CFIRST>
__global__ __launch_bounds__(WG) void k_rows_scan_apply(T *a, long n, const T *part, int *cfirst, int m, int *hnnz) {
    __shared__ T tile[RS_TILE + RS_TILE / 16];
    __shared__ T red[WAVES];
    const int tid = threadIdx.x;
    const long base = (long)blockIdx.x * RS_TILE;
    T pre = 0;
    for (int i = tid; i < (int)blockIdx.x; i += WG) pre += part[i];
#pragma unroll
    for (int u = 0; u < RS_ITEMS; ++u) {
        const int li = u * WG + tid;
        const long i = base + li;
        tile[rs_pad(li)] = i < n ? a[i] : T(0);
    }
    pre = block_sum(pre, red);  // (its barriers also publish the tile)
    T sum = 0;
#pragma unroll
    for (int u = 0; u < RS_ITEMS; ++u) sum += tile[rs_pad(tid * RS_ITEMS + u)];
    T tot;
    T off = block_excl_scan(sum, &tot, red) + pre;
#pragma unroll
    for (int u = 0; u < RS_ITEMS; ++u) {
        const int li = rs_pad(tid * RS_ITEMS + u);
        const T v = tile[li];
        tile[li] = off;
        if constexpr (CFIRST) {
            const long r = base + tid * RS_ITEMS + u;
            if (r < m) {
                if (cfirst)
                    for (long long b = ((long long)off + CP_CH - 1) / CP_CH; b * CP_CH < (long long)off + v; ++b)
                        cfirst[b] = (int)r;
            } else if (r == m && hnnz) {
                __hip_atomic_store(hnnz, (int)off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        off += v;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < RS_ITEMS; ++u) {
        const int li = u * WG + tid;
        const long i = base + li;
        if (i < n) a[i] = tile[rs_pad(li)];
    }
}

__device__ __forceinline__ int row_class(long long P, int k) {
    if (P == 0) return -1;
    if (P <= S16_MAX && k <= S16_MAX) return 0;
    if (P <= RS_MAX && k <= RS_MAX) return 1;
    if (P <= M0_CAP && k <= M0_RUNS) return 2;
    if (P <= M1_CAP && k <= M1_RUNS) return 3;
    if (P <= M2_CAP && k <= M2_RUNS) return 4;
    if (P <= M3_CAP && k <= M3_RUNS) return 5;
    if (P <= M4_CAP && k <= M4_RUNS) return 6;
    return 7;
}

// rows -> classes: lists (class c's rows from lists + c*m) and counts cls[0..NCLS);
// rows without products get nnz 0; hst[0] = the class-H rows' products, hst[1]
// = the largest row's products (the routing statistics), hst[2] = all products,
// hst[3] = the products of hub rows (past kRowsHubProducts), hst[4] = the
// class-H rows with more than OW_RUNS runs, hst[8] = the class-H rows'
// products past OW_CH (the one-walk rows' scratch)
// (*Etot, copied so that one read-back brings everything); rnnz[m] = 0 (the
// row pointers' n+1 slot).  A workgroup per
// BIN_ROWS rows: its counts first (one atomic per class), then its rows in
// order into the reserved slots.
__global__ __launch_bounds__(WG) void k_rows_bin(const int *rpA, int m, const long long *E, const long long *Etot,
                                                 int *rnnz, int4 *lists, int *cls, long long *soff,
                                                 unsigned long long *hst, const int *spart, int snb, int *sflag) {
    __shared__ int gb[NCLS];
    __shared__ long long red64[WAVES];
    constexpr int RPT = BIN_ROWS / WG;  // rows per thread: every load of a sweep issued together
    __shared__ int wcu[RPT][NCLS][WAVES];  // per (row slot, class, wave): count, then exclusive prefix
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int r0 = blockIdx.x * BIN_ROWS, r1 = min(m, r0 + BIN_ROWS);
    if (blockIdx.x == 0 && tid == 0) {
        hst[2] = (unsigned long long)*Etot;
        rnnz[m] = 0;
    }
    if (blockIdx.x == 0 && spart) {  // B's sortedness: the shares' sum (dev_rows_sorted_shares)
        long long v = 0;  // (<= 4,096 shares: SRT_MAXB)
#pragma unroll 8
        for (int i = tid; i < snb; i += WG) v += spart[i];
        v = block_sum(v, red64);
        if (tid == 0 && v != 0) __hip_atomic_store(sflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    long long hp = 0, pmax = 0, drp = 0, hubr = 0, hbig = 0;
    int cu[RPT];  // each of the thread's rows' class (-1: none)
    int ra0[RPT], ra1[RPT];
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int r = r0 + u * WG + tid;
        ra0[u] = r < r1 ? rpA[r] : 0;
        ra1[u] = r < r1 ? rpA[r + 1] : 0;
    }
    long long e0[RPT], e1[RPT];
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        e0[u] = E[ra0[u]];
        e1[u] = E[ra1[u]];
    }
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int r = r0 + u * WG + tid;
        cu[u] = -1;
        if (r >= r1) continue;
        const long long P = e1[u] - e0[u];
        const int c = row_class(P, ra1[u] - ra0[u]);
        soff[r] = e0[u];  // the row's staging offset
        cu[u] = c;
        if (c < 0) rnnz[r] = 0;
        hp += c == NCLS - 1 ? P : 0;
        hbig += c == NCLS - 1 && P <= kRowsHubProducts && P > OW_CH ? P - OW_CH : 0;
        pmax = max(pmax, P);
        // hub rows (the DR or windowed kernels decide which, k_rows_wplan) and
        // class-H rows with more runs than the one-walk kernel takes
        if (P > kRowsHubProducts) drp += P;
        if (c == NCLS - 1 && ra1[u] - ra0[u] > OW_RUNS) ++hubr;
    }
    hp = block_sum(hp, red64);
    drp = block_sum(drp, red64);
    hubr = block_sum(hubr, red64);
    hbig = block_sum(hbig, red64);
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) pmax = max(pmax, __shfl_xor(pmax, d, 64));
    if (lane == 0) red64[wv] = pmax;
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < WAVES; ++w) pmax = max(pmax, red64[w]);
        if (hp) atomicAdd(&hst[0], (unsigned long long)hp);
        if (pmax) atomicMax(&hst[1], (unsigned long long)pmax);
        if (drp) atomicAdd(&hst[3], (unsigned long long)drp);
        if (hubr) atomicAdd(&hst[4], (unsigned long long)hubr);
        if (hbig) atomicAdd(&hst[8], (unsigned long long)hbig);
    }
    // the list slots with two barriers (one sweep per row slot u had cost two
    // each: 16 on a workgroup of 8 row slots): per (u, class) each wave's count
    // by a ballot; eight threads turn them into exclusive prefixes in (u, wave)
    // order and reserve each class's run of slots with one atomic
    u64 mine[RPT];  // the ballot of this lane's class, per row slot
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        mine[u] = 0;
#pragma unroll
        for (int t = 0; t < NCLS; ++t) {
            const u64 bt = __ballot(cu[u] == t);
            if (cu[u] == t) mine[u] = bt;
            if (lane == 0) wcu[u][t][wv] = __popcll(bt);
        }
    }
    __syncthreads();
    if (tid < NCLS) {
        int run = 0;
        for (int u = 0; u < RPT; ++u)
            for (int w = 0; w < WAVES; ++w) {
                const int v = wcu[u][tid][w];
                wcu[u][tid][w] = run;
                run += v;
            }
        gb[tid] = run ? atomicAdd(&cls[tid], run) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int c = cu[u];
        if (c >= 0) {
            const int r = r0 + u * WG + tid;
            lists[(long)c * m + gb[c] + wcu[u][c][wv] + lanes_below(mine[u])] = make_int4(r, ra0[u], ra1[u] - ra0[u], 0);
        }
    }
}

// class H's rows longest first (products in buckets of 1,024, a counting sort
// in one workgroup): the dispatch order is the list order, and a long row
// started last set the class's tail (row order: ~30 % over the longest-first
// makespan on webbase).  Past OH_MAX rows the list keeps row order.
constexpr int OH_NT = 1024, OH_PER = 8, OH_MAX = OH_NT * OH_PER, OH_NB = 64;
__global__ __launch_bounds__(OH_NT) void k_rows_order_h(const long long *E, const int *cls, int4 *list) {
    __shared__ int cnt[OH_NB];
    const int tid = threadIdx.x;
    const int n = cls[NCLS - 1];
    if (n < 2 || n > OH_MAX) return;  // (workgroup-uniform)
    if (tid < OH_NB) cnt[tid] = 0;
    __syncthreads();
    int4 r[OH_PER];
    int b[OH_PER];
#pragma unroll
    for (int u = 0; u < OH_PER; ++u) {
        const int i = u * OH_NT + tid;
        r[u] = i < n ? list[i] : make_int4(-1, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < OH_PER; ++u)
        if (r[u].x >= 0) {
            const long long P = E[r[u].y + r[u].z] - E[r[u].y];
            b[u] = OH_NB - 1 - (int)min((long long)OH_NB - 1, P >> 10);  // longest first
            atomicAdd(&cnt[b[u]], 1);
        }
    __syncthreads();
    if (tid < 64) {
        const int v = cnt[tid];
        const int inc = wave_incl_scan_dpp(v);
        cnt[tid] = inc - v;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < OH_PER; ++u)
        if (r[u].x >= 0) list[atomicAdd(&cnt[b[u]], 1)] = r[u];
}

// lane J of each row of 16 lanes, to every lane of that row: DPP row_newbcast
// (a VALU move; __shfl inside 16 lanes is a ds_bpermute on the LDS pipe, and
// the S16 kernel's rank loop issued 48 of them per row)
template <int J> __device__ __forceinline__ int row_bcast16(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 | J, 0xf, 0xf, false);
}
template <int V> struct IntC { static constexpr int value = V; };
template <int J, int N, class F> __device__ __forceinline__ void static_for(F &&f) {
    if constexpr (J < N) {
        f(IntC<J>{});
        static_for<J + 1, N>(f);
    }
}

// ---- classes S16 / S64: G lanes per row (64/G rows per wave), the products
// one per lane, ranks by counting the group's smaller (column, lane) keys.
// Each lane group takes U rows: the rows' loads (list, entries, B) are issued
// stage by stage for all U together, so a wave waits for three dependent
// memory round trips per U rows rather than per row (the classes are bound by
// those chains, not by bytes: 85 us for mc2depi's 0.5 M S16 rows at U = 1).
template <int G, int U>
__global__ __launch_bounds__(WG) void k_rows_small(RowsArgs g) {
    constexpr int RPW = 64 / G;
    __shared__ u64 sk[WAVES][U][64];
    __shared__ double sv[WAVES][U][64];
    const int lane = lane_id(), wv = wave_id(), sl = lane % G, gb = lane - sl;
    const int w0 = (blockIdx.x * WAVES + wv) * RPW * U;  // the wave's first row
    if (w0 >= g.nrows) return;                           // wave-uniform
    int r[U], a0[U], k[U];
    bool live[U];
    long long base[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = w0 + u * RPW + lane / G;
        live[u] = i < g.nrows;
        r[u] = 0, a0[u] = 0, k[u] = 0;
        if (live[u]) {
            const int4 e = g.list[i];
            r[u] = e.x;
            a0[u] = e.y;
            k[u] = e.z;
        }
    }
    // lane sl < k: run sl's B range and A value (and the row's output offset)
    int2 be[U];
    double av[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        be[u] = make_int2(0, 0);
        av[u] = 0.0;
        base[u] = 0;
        if (live[u]) base[u] = g.E[a0[u]];  // (not waited for until the output)
        if (sl < k[u]) {
            be[u] = g.ebnd[a0[u] + sl];
            av[u] = g.vA[a0[u] + sl];
        }
    }
    // the runs' offsets in each row by a scan of their lengths over the group;
    // position sl's run = the last run starting at or before it; its B element
    int P[U], pp[U];
    double ra[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int len = be[u].y - be[u].x, bs = be[u].x;
        int inc = len;  // inclusive scan over the G lanes (DPP row shifts stay inside 16-lane rows)
        inc += dpp_mov<0x111, 0xf>(0, inc);
        inc += dpp_mov<0x112, 0xf>(0, inc);
        inc += dpp_mov<0x114, 0xf>(0, inc);
        inc += dpp_mov<0x118, 0xf>(0, inc);
        if constexpr (G == 64) {
            inc += dpp_mov<0x142, 0xa>(0, inc);  // row_bcast:15
            inc += dpp_mov<0x143, 0xc>(0, inc);  // row_bcast:31
        }
        const int roff = sl < k[u] ? inc - len : INT_MAX;
        int run = 0;
        if constexpr (G == 64) {
            P[u] = __shfl(inc, G - 1, G);
            for (int j = 1; j < k[u]; ++j) run = (__builtin_amdgcn_readlane(roff, j) <= sl) ? j : run;
        } else {
            static_assert(G == 16, "row broadcasts: 16-lane groups");
            P[u] = row_bcast16<15>(inc);
            static_for<1, 16>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                run = row_bcast16<j>(roff) <= sl ? j : run;
            });
        }
        const int rs = __shfl(roff, run, G), rb = __shfl(bs, run, G);
        ra[u] = __shfl(av[u], run, G);
        pp[u] = rb + sl - rs;
    }
    u64 key[U];
    double x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        key[u] = ~0ull;
        x[u] = 0.0;
        if (sl < P[u]) {
            key[u] = ((u64)(u32)g.Bcol[pp[u]] << 32) | (u32)sl;
            x[u] = g.Bval[pp[u]];
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32 khi = (u32)(key[u] >> 32), klo = (u32)key[u];
        int rank = 0;
        if constexpr (G == 64) {  // one row per wave: P is wave-uniform, scalar reads of each key
            for (int f = 0; f < P[u]; ++f) {
                const u64 kf = ((u64)(u32)__builtin_amdgcn_readlane((int)khi, f) << 32) |
                               (u32)__builtin_amdgcn_readlane((int)klo, f);
                rank += kf < key[u];
            }
        } else {
            const u64 ku = key[u];
            static_for<0, 16>([&](auto fc) {
                constexpr int f = decltype(fc)::value;
                const u64 kf = ((u64)(u32)row_bcast16<f>((int)khi) << 32) | (u32)row_bcast16<f>((int)klo);
                rank += kf < ku;  // (lanes past P hold ~0: never below a product)
            });
        }
        if (sl < P[u]) {
            sk[wv][u][gb + rank] = key[u];
            sv[wv][u][gb + rank] = ra[u] * x[u];
        }
    }
    wave_lds_sync();
    const u64 gm = (G == 64 ? ~0ull : ((1ull << (G & 63)) - 1ull)) << gb;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int col = -1;
        bool head = false;
        if (sl < P[u]) {
            col = key_col(sk[wv][u][gb + sl]);
            head = sl == 0 || key_col(sk[wv][u][gb + sl - 1]) != col;
        }
        const u64 hb = __ballot(head) & gm;
        if (head) {
            double sm = sv[wv][u][gb + sl];
            for (int j = sl + 1; j < P[u] && key_col(sk[wv][u][gb + j]) == col; ++j) sm += sv[wv][u][gb + j];
            const long long o = base[u] + (long long)lanes_below(hb);
            g.Scol[o] = col;
            g.Sval[o] = sm;
        }
        if (live[u] && sl == 0) g.rnnz[r[u]] = __popcll(hb);
    }
}

// U independent searches in lockstep (U LDS reads in flight per step): first
// index in [b, b + len) whose element is >= key (or > key where ub[u])
template <int U, class T>
__device__ __forceinline__ void search_ilp(const T *a, int (&b)[U], int (&len)[U], const T (&key)[U],
                                           const bool (&ub)[U]) {
    for (;;) {
        bool more = false;
#pragma unroll
        for (int u = 0; u < U; ++u) more |= len[u] > 0;
        if (!more) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int half = len[u] >> 1, idx = b[u] + half;
            const T v = a[len[u] > 0 ? idx : 0];  // (finished searches: one broadcast address)
            const bool go = len[u] > 0 && (v < key[u] || (ub[u] && v == key[u]));
            b[u] = go ? idx + 1 : b[u];
            len[u] = go ? len[u] - half - 1 : half;
        }
    }
}

// lane l's value of lane l ^ D (D a power of two below 64): DPP quad
// permutes for 1 and 2, ds_swizzle's xor mode inside 32 lanes, ds_bpermute for 32
template <int D> __device__ __forceinline__ u32 lane_xor(u32 v) {
    if constexpr (D == 1) return (u32)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);  // [1,0,3,2]
    else if constexpr (D == 2) return (u32)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // [2,3,0,1]
    else if constexpr (D < 32) return (u32)__builtin_amdgcn_ds_swizzle((int)v, (D << 10) | 0x1f);
    else return (u32)__shfl_xor((int)v, D, 64);
}

// one bitonic stage at element distance J inside sequences of K (elements
// e = 4*lane + u): ascending where e & K == 0
// (compare-exchanges whose direction varies by lane: one compare, the
// direction folded into the lane mask, one select -- instead of min, max and a
// select per element)
template <int K, int J> __device__ __forceinline__ void bitonic_stage(u32 (&x)[4], int lane) {
    if constexpr (J >= 4) {
        constexpr int D = J / 4;
        const bool asc = K >= 256 || (lane & (K / 4)) == 0;
        const bool keep_max = asc != ((lane & D) == 0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const u32 y = lane_xor<D>(x[u]);
            x[u] = ((y < x[u]) != keep_max) ? y : x[u];
        }
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if ((u & J) == 0) {
                if constexpr (K < 4 || K >= 256) {  // the direction is the same on every lane
                    const bool asc = K < 4 ? (u & K) == 0 : true;  // (u: unrolled, a constant)
                    const u32 lo = min(x[u], x[u + J]), hi = max(x[u], x[u + J]);
                    x[u] = asc ? lo : hi;
                    x[u + J] = asc ? hi : lo;
                } else {
                    const bool desc = (lane & (K / 4)) != 0;
                    const bool sw = (x[u + J] < x[u]) != desc;
                    const u32 a = x[u], b = x[u + J];
                    x[u] = sw ? b : a;
                    x[u + J] = sw ? a : b;
                }
            }
    }
}
template <int K, int J> __device__ __forceinline__ void bitonic_merge(u32 (&x)[4], int lane) {
    bitonic_stage<K, J>(x, lane);
    if constexpr (J > 1) bitonic_merge<K, J / 2>(x, lane);
}
template <int K> __device__ __forceinline__ void bitonic_sort(u32 (&x)[4], int lane) {
    if constexpr (K > 2) bitonic_sort<K / 2>(x, lane);
    bitonic_merge<K, K / 2>(x, lane);
}
// a wave's 256 keys ascending in registers, lane l holding elements 4l..4l+3
// (36 compare-exchange stages, 21 of them across lanes; no LDS, no barrier)
__device__ __forceinline__ void wave_sort256(u32 (&x)[4], int lane) { bitonic_sort<256>(x, lane); }

// ---- classes M0..M4: a row's runs sorted into one column-ordered sequence in
// LDS.  NT threads per row, at most CAP products and RUNS A entries (so a
// thread per entry).
//
// The expansion loads each product's B column AND value together (one round
// trip): the value a*b goes to LDS in expansion order, and after the sort
// each key's low bits (its expansion position) find it there -- no second
// dependent gather of B's values after the sort.
//
// Keys: when the row's column span fits, one u32 per element packs
// (column - lo, expansion position) -- unique, so the sorted order is one fixed
// order and every sum is taken in it.  Each wave sorts its 256 positions in
// registers with a bitonic network, then the rest of a bitonic sort over the
// waves' segments runs through LDS.  Wider rows sort u32 columns with a
// (run, position) payload by merge-path rounds, ties from the left group first
// (equal columns stay in run order), and reload their values after.
template <int NT, int CAP, int RUNS>
__global__ __launch_bounds__(NT, NT == 1024 ? 8 : 1) void k_rows_merge(RowsArgs g) {
    constexpr int NW = NT / 64;
    constexpr int IPM = (CAP + NT - 1) / NT | 1;
    constexpr int IB = CAP == 256 ? 8 : CAP == 512 ? 9 : CAP == 1024 ? 10 : CAP == 2048 ? 11 : 12;  // position bits
    static_assert((1 << IB) == CAP, "CAP: a power of two in [256, 4096]");
    constexpr int SEG = 256;
    static_assert(CAP == 4 * NT, "four positions per thread");
    static_assert(RUNS <= NT, "a thread per A entry");
    // packed: keys ping-pong kp[0][0] <-> kp[0][1], the values (expansion
    // order) in kp[1] as CAP doubles.  Unpacked: [buffer][keys | payloads],
    // the values gathered at the end into the free buffer.
    __shared__ __align__(16) u32 kp[2][2][CAP];
    __shared__ int roff[RUNS + 1];
    __shared__ int rbs[RUNS];       // each run's B start
    __shared__ double rav[RUNS];    // each run's A value
    __shared__ int red[2 * NW];
    RP_INIT
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int4 le = g.list[blockIdx.x];
    int2 be = make_int2(0, 0);
    double av = 0.0;
    if (tid < le.z) {
        be = g.ebnd[le.y + tid];
        av = g.vA[le.y + tid];
    }
    const long long base = g.E[le.y];  // (the output offset: not waited for until the output)
    double *const V = reinterpret_cast<double *>(kp[1][0]);
    {
        const int r = le.x;
        // the runs with products, in order (entries selecting empty B rows
        // dropped: fewer runs); their offsets by a scan of the B row lengths
        int k = 0, P = 0;
        {
            const int len = be.y - be.x;
            const u64 b = __ballot(len > 0);
            const int inc = wave_incl_scan_dpp(len);
            if (lane == 63) {
                red[wv] = __popcll(b);
                red[NW + wv] = inc;
            }
            __syncthreads();
            int off = 0, loff = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                off += w < wv ? red[w] : 0;
                k += red[w];
                loff += w < wv ? red[NW + w] : 0;
                P += red[NW + w];
            }
            if (len > 0) {
                const int d = off + lanes_below(b);
                roff[d] = loff + inc - len;
                rbs[d] = be.x;
                rav[d] = av;
            }
            if (tid == 0) roff[k] = P;
            __syncthreads();
        }
        RP(0);
        // expansion: wave w takes positions [256w, 256w + 256), lane l the four at
        // e0 = 256w + 4l (mostly one run's neighbours); position q of run j at
        // roff[j] + t -> column, value, payload (j, t)
        const int e0 = wv * SEG + 4 * lane, ne = max(0, min(4, P - e0));
        int c[4] = {0, 0, 0, 0};
        u32 py[4] = {0, 0, 0, 0};
        double xv[4] = {0.0, 0.0, 0.0, 0.0};
        {
            int j = 0;
            if (ne > 0) j = lower_bound_dev(roff, 0, k + 1, e0 + 1) - 1;  // the last run starting at or before e0
            int pa[4] = {0, 0, 0, 0};
            double ra[4] = {0.0, 0.0, 0.0, 0.0}, bv[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (u < ne) {
                    const int q = e0 + u;
                    while (roff[j + 1] <= q) ++j;
                    pa[u] = rbs[j] + q - roff[j];
                    py[u] = ((u32)j << 16) | (u32)(q - roff[j]);
                    ra[u] = rav[j];
                }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (u < ne) {
                    c[u] = g.Bcol[pa[u]];
                    bv[u] = g.Bval[pa[u]];
                }
#pragma unroll
            for (int u = 0; u < 4; ++u) xv[u] = u < ne ? ra[u] * bv[u] : 0.0;
        }
        // the row's column span [clo, chi]
        int clo = INT_MAX, chi = -1;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (u < ne) {
                clo = min(clo, c[u]);
                chi = max(chi, c[u]);
            }
        clo = wave_last(wave_incl_dpp(clo, INT_MAX, OpMin{}));
        chi = wave_last(wave_incl_dpp(chi, INT_MIN, OpMax{}));
        if (lane == 0) {
            red[wv] = clo;
            red[NW + wv] = chi;
        }
        __syncthreads();
        clo = red[0];
        chi = red[NW];
#pragma unroll
        for (int w = 1; w < NW; ++w) {
            clo = min(clo, red[w]);
            chi = max(chi, red[NW + w]);
        }
        // (strict: the largest packed key stays below the ~0u padding)
        const bool packed = (u32)(chi - clo) < (1u << (32 - IB)) - 1u;  // (workgroup-uniform)
        int npow = SEG;  // the packed sort's length: P padded to a power of two (with ~0u keys)
        while (npow < P) npow <<= 1;
        u32 x[4] = {~0u, ~0u, ~0u, ~0u};  // packed: this lane's four keys
        if (packed) {
            // each wave sorts its 256 positions in registers: the LDS stages
            // start from sorted segments of 256
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = u < ne ? ((u32)(c[u] - clo) << IB) | (u32)(e0 + u) : ~0u;
            if (ne > 0) {
                reinterpret_cast<double4 *>(V)[e0 >> 2] = make_double4(xv[0], xv[1], xv[2], xv[3]);
            }
            if (wv * SEG < P) wave_sort256(x, lane);  // (wave-uniform)
            if (wv * SEG < npow) *reinterpret_cast<uint4 *>(kp[0][0] + e0) = make_uint4(x[0], x[1], x[2], x[3]);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (u < ne) {
                    kp[0][0][e0 + u] = (u32)c[u];
                    kp[0][1][e0 + u] = py[u];
                }
        }
        __syncthreads();
        RP(1);
        int src = 0;  // packed: the key buffer holding the (merged) keys
        if (packed) {
            // the waves' sorted segments merged by the rest of a bitonic sort over
            // npow keys, every sequence ascending: per level K the first stage pairs
            // each position with its mirror in the K-block (e ^ (K-1)), the stages
            // at distances K/4 .. 256 pair across waves through LDS (uint4 per
            // lane, the two key buffers in turn, one barrier each), the last eight
            // stay in registers.
            const bool act = wv * SEG < npow;  // (wave-uniform)
            auto cmpx = [&](const uint4 y, bool rev, bool keep_min) {
                const u32 yy[4] = {rev ? y.w : y.x, rev ? y.z : y.y, rev ? y.y : y.z, rev ? y.x : y.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) x[u] = keep_min ? min(x[u], yy[u]) : max(x[u], yy[u]);
            };
            for (int K = 2 * SEG; K <= npow; K <<= 1) {  // (workgroup-uniform)
                if (act) cmpx(*reinterpret_cast<const uint4 *>(kp[0][src] + (e0 ^ (K - 4))), true, (e0 & (K >> 1)) == 0);
                for (int J = K >> 2; J >= SEG; J >>= 1) {
                    src ^= 1;
                    if (act) *reinterpret_cast<uint4 *>(kp[0][src] + e0) = make_uint4(x[0], x[1], x[2], x[3]);
                    __syncthreads();
                    if (act) cmpx(*reinterpret_cast<const uint4 *>(kp[0][src] + (e0 ^ J)), false, (e0 & J) == 0);
                }
                if (act) bitonic_merge<256, 128>(x, lane);
                src ^= 1;
                if (act) *reinterpret_cast<uint4 *>(kp[0][src] + e0) = make_uint4(x[0], x[1], x[2], x[3]);
                __syncthreads();
            }
        }
        // unpacked rows: merge-path rounds from the runs; thread t owns
        // [t*ipt, t*ipt + ipt) of every round
        const int ipt = ((P + NT - 1) / NT) | 1;
        const int q0 = min(P, tid * ipt), q1 = min(P, q0 + ipt), nq = q1 - q0;
        if (!packed) {
            const int *const bd = roff;
            const int nb = k;
            int j0 = 0;  // the group holding q0 (pairs keep their position ranges every round)
            if (nq > 0) j0 = lower_bound_dev(roff, 0, k + 1, q0 + 1) - 1;
            for (int lw = 0; (1 << lw) < nb; ++lw) {  // groups of 2^lw runs merged pairwise
                const u32 *ik = kp[src][0], *ip = kp[src][1];
                u32 *ok = kp[src ^ 1][0], *op = kp[src ^ 1][1];
                int pr = j0 >> (lw + 1);  // the pair holding q0
                for (int q = q0; q < q1;) {
                    while (bd[min((pr + 1) << (lw + 1), nb)] <= q) ++pr;  // (pairs ending at or before q)
                    const int ps = bd[pr << (lw + 1)];
                    const int pm = bd[min((2 * pr + 1) << lw, nb)];
                    const int pe = bd[min((pr + 1) << (lw + 1), nb)];
                    const int la = pm - ps, lb = pe - pm, qq = q - ps;
                    int lo = max(0, qq - lb), hi = min(qq, la);
                    while (lo < hi) {
                        const int t = (lo + hi) >> 1;
                        if (ik[ps + t] <= ik[pm + qq - t - 1]) lo = t + 1; else hi = t;
                    }
                    int ia = lo, ib = qq - lo;
                    u32 ka = ia < la ? ik[ps + ia] : ~0u, kbv = ib < lb ? ik[pm + ib] : ~0u;  // (keys < 2^32 - 1)
                    const int qe = min(q1, pe);
                    for (; q < qe; ++q) {  // one dependent LDS read per output
                        const bool ta = ka <= kbv;
                        ok[q] = ta ? ka : kbv;
                        op[q] = ta ? ps + ia : pm + ib;  // (the source position, for now)
                        ia += ta;
                        ib += !ta;
                        const u32 kn = ik[ta ? ps + ia : pm + ib];  // (an exhausted side reads a neighbour: masked)
                        const bool live = ta ? ia < la : ib < lb;
                        ka = ta ? (live ? kn : ~0u) : ka;
                        kbv = ta ? kbv : (live ? kn : ~0u);
                    }
                }
#pragma unroll
                for (int u = 0; u < IPM; ++u)  // the payloads: independent reads
                    if (u < nq) op[q0 + u] = ip[op[q0 + u]];
                __syncthreads();
                src ^= 1;
            }
        }
        RP(2);
        // heads (first position of each column) and the values in sorted order
        int nh = 0;
        const int np = packed ? max(0, min(4, P - e0)) : 0;
        double xs[4] = {0.0, 0.0, 0.0, 0.0};
        u32 hd = 0;  // packed: head bits of the four positions
        const u32 *const sk = packed ? kp[0][src] : kp[src][0];
        double *const vb = reinterpret_cast<double *>(kp[src ^ 1][0]);  // unpacked: the free buffer
        if (packed) {
            const u32 prev = e0 > 0 && np > 0 ? sk[e0 - 1] : ~0u;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (u < np) {
                    xs[u] = V[x[u] & (CAP - 1)];
                    const u32 pk = u ? x[u - 1] : prev;
                    hd |= (e0 + u == 0 || (x[u] >> IB) != (pk >> IB)) ? 1u << u : 0u;
                }
            nh = __popc(hd);
        } else {
            const u32 *sp = kp[src][1];
            int pa[IPM] = {};
            double ra[IPM] = {};
#pragma unroll
            for (int u = 0; u < IPM; ++u)
                if (u < nq) {
                    const u32 key = sk[q0 + u];
                    const u32 pj = sp[q0 + u];
                    const int ru = (int)(pj >> 16);
                    pa[u] = rbs[ru] + (int)(pj & 0xffffu);
                    ra[u] = rav[ru];
                    nh += (q0 + u == 0 || key != sk[q0 + u - 1]);
                }
            double xx[IPM] = {};
#pragma unroll
            for (int u = 0; u < IPM; ++u)
                if (u < nq) xx[u] = ra[u] * g.Bval[pa[u]];
#pragma unroll
            for (int u = 0; u < IPM; ++u)
                if (u < nq) vb[q0 + u] = xx[u];
        }
        // the chunk's first output slot: exclusive scan of the head counts
        const int inc = wave_incl_scan_dpp(nh);
        if (lane == 63) red[wv] = inc;
        __syncthreads();
        RP(3);
        int o = inc - nh, tot = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            o += w < wv ? red[w] : 0;
            tot += red[w];
        }
        if (tid == 0) g.rnnz[r] = tot;
        if (packed) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (hd >> u & 1u) {
                    const u32 col = x[u] >> IB;
                    double sum = xs[u];
                    int j = u + 1;
#pragma unroll
                    for (int v = u + 1; v < 4; ++v)  // (ascending, as below: deterministic)
                        if (j == v && v < np && (x[v] >> IB) == col) {
                            sum += xs[v];
                            ++j;
                        }
                    if (j == 4)
                        for (int q = e0 + 4; q < P && (sk[q] >> IB) == col; ++q) sum += V[sk[q] & (CAP - 1)];
                    g.Scol[base + o] = (int)col + clo;
                    g.Sval[base + o] = sum;
                    ++o;
                }
        } else {
            for (int q = q0; q < q1; ++q) {
                const u32 col = sk[q];
                if (q == 0 || sk[q - 1] != col) {
                    double sum = vb[q];
                    for (int j = q + 1; j < P && sk[j] == col; ++j) sum += vb[j];  // ascending: deterministic
                    g.Scol[base + o] = (int)col;
                    g.Sval[base + o] = sum;
                    ++o;
                }
            }
        }
        RP(4);
    }
    RP_DONE(CAP <= M1_CAP ? 2 : 1);  // (M0, M1 | M2..M4)
}

// ---- class H: a workgroup per row; windows of RH_SPAN columns, each a bitmap
// in LDS.  The row's products are walked in batches of RH_NT runs (a thread per
// run: lengths scanned over the workgroup, then the batch's products flattened
// over all threads, U at a time).
struct WalkTab {
    int pre[RH_NT];     // products before each run of the batch
    int bs[RH_NT];      // B start
    double av[RH_NT];   // A value
    int red[RH_NT / 64];
    int tot;            // the batch's products
};
// a batch's run table (thread per run; lengths scanned over the workgroup)
__device__ __forceinline__ void rows_batch(const RowsArgs &g, int a0, int k, int b0, WalkTab &tb) {
    constexpr int NW = RH_NT / 64;
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int j = b0 + tid;
    int2 be = make_int2(0, 0);
    double av = 0.0;
    if (j < k) {
        be = g.ebnd[a0 + j];
        av = g.vA[a0 + j];
    }
    const int len = be.y - be.x;
    const int inc = wave_incl_scan_dpp(len);
    if (lane == 63) tb.red[wv] = inc;
    __syncthreads();
    int woff = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const int v = tb.red[w];
        woff += w < wv ? v : 0;
        tot += v;
    }
    tb.pre[tid] = woff + inc - len;
    tb.bs[tid] = be.x;
    tb.av[tid] = av;
    if (tid == 0) tb.tot = tot;
    __syncthreads();
}
// the run of every product of [qb, qb + 4 * RH_NT) into rmap (u16; the batch's
// nb runs in tb): each run marks its first product there, a workgroup
// max-scan fills the rest (runs ascend with the products).  One LDS read per
// product afterwards instead of a binary search of the run table.  Every
// thread calls it (barriers); red: RH_NT / 64 ints.
__device__ __forceinline__ void batch_runmap(const WalkTab &tb, int nb, int qb, unsigned short *rmap, int *red) {
    constexpr int NW = RH_NT / 64;
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    reinterpret_cast<uint2 *>(rmap)[tid] = make_uint2(0u, 0u);
    __syncthreads();
    if (tid < nb) {
        const int p0 = tb.pre[tid], p1 = tid + 1 < nb ? tb.pre[tid + 1] : tb.tot;
        if (p1 > p0 && p1 > qb && p0 < qb + 4 * RH_NT) rmap[max(p0, qb) - qb] = (unsigned short)tid;
    }
    __syncthreads();
    uint2 v = reinterpret_cast<const uint2 *>(rmap)[tid];
    int m[4];
    m[0] = (int)(v.x & 0xffffu);
    m[1] = max(m[0], (int)(v.x >> 16));
    m[2] = max(m[1], (int)(v.y & 0xffffu));
    m[3] = max(m[2], (int)(v.y >> 16));
    const int inc = wave_incl_dpp(m[3], 0, OpMax{});
    if (lane == 63) red[wv] = inc;
    int carry = __shfl_up(inc, 1, 64);
    if (lane == 0) carry = 0;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NW; ++w) carry = w < wv ? max(carry, red[w]) : carry;
    v.x = (u32)max(m[0], carry) | ((u32)max(m[1], carry) << 16);
    v.y = (u32)max(m[2], carry) | ((u32)max(m[3], carry) << 16);
    reinterpret_cast<uint2 *>(rmap)[tid] = v;
    __syncthreads();
}

// products [q0, q1) of a batch whose run table tb holds (rows_batch; nb runs),
// U per thread at a time: each product's column (and with VAL its a*b) to
// f(column, value, valid), called by every lane (consecutive lanes hold
// consecutive products; the invalid ones are a suffix of the wave).  Each
// step's runs come from batch_runmap (rmap: two maps of 4 * RH_NT u16, red:
// every thread must call).  Software-pipelined: step s + 1's map is built and
// its B loads issued before f runs on step s, so the loads are in flight
// through f (its LDS atomics and stores); the maps alternate, so a map is
// rebuilt only after a barrier past its last reads.  (One step at a time --
// map, loads, wait, f -- left the memory pipe idle through the map's barriers
// and f: 856 us of k_rows_wscatter on the LiveJournal block, r5p.)
template <bool VAL, class F>
__device__ __forceinline__ void batch_walk(const RowsArgs &g, int nb, int q0, int q1, const WalkTab &tb, F &&f,
                                           unsigned short *rmap, int *red) {  // (q1 - q0 <= W_CH)
    constexpr int U = 4;
    const int tid = threadIdx.x;
    if (q0 >= q1) return;  // (workgroup-uniform)
    int c[U], cn[U];
    double x[U], xn[U];
    // step qb's products: its map into rm, then every load issued -- unconditional
    // (invalid lanes read B's first entry) and raw, the a*b product taken at use:
    // a load under a branch, or arithmetic on it here, makes hipcc wait for it here
    auto fetch = [&](int qb, unsigned short *rm, int (&cc)[U], double (&xx)[U]) {
        __syncthreads();  // (the last use of the map rm held, two steps back, done everywhere)
        batch_runmap(tb, nb, qb, rm, red);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = qb + u * RH_NT + tid;
            const int r = q < q1 ? rm[u * RH_NT + tid] : 0;
            const int bs = tb.bs[r], pre = tb.pre[r];
            const int pp = q < q1 ? bs + q - pre : 0;
            cc[u] = g.Bcol[pp];
            if (VAL) xx[u] = g.Bval[pp];
        }
    };
    // the run of each product read again from its step's map at use (the map is
    // rebuilt only by the fetch after this use): no register set of runs
    auto use = [&](int qb, const unsigned short *rm, const int (&cc)[U], const double (&xx)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {  // (every lane: f may use wave operations)
            const bool ok = qb + u * RH_NT + tid < q1;
            f(cc[u], VAL && ok ? tb.av[rm[u * RH_NT + tid]] * xx[u] : 0.0, ok);
        }
    };
    constexpr int STEP = U * RH_NT;
    // two register sets, fully unrolled over the at most W_CH / STEP steps of a
    // chunk: straight-line code, where hipcc counts the waits exactly (in a loop,
    // its register moves on the back edge waited for the set still loading); each
    // fetch unconditional -- past q1 its lanes all read B's first entry -- so that
    // no path leaves a set's loads the latest
    unsigned short *const rm0 = rmap, *const rm1 = rmap + 4 * RH_NT;
    fetch(q0, rm0, c, x);
#pragma unroll
    for (int st = 0; st < W_CH / STEP; st += 2) {  // (workgroup-uniform)
        const int qb = q0 + st * STEP;
        if (qb >= q1) break;
        fetch(qb + STEP, rm1, cn, xn);
        use(qb, rm0, c, x);
        if (qb + STEP >= q1) break;
        fetch(qb + 2 * STEP, rm0, c, x);
        use(qb + STEP, rm1, cn, xn);
    }
}

// ranks inside a window: blk[w / RH_BLK] + g4[w / 4] + the bits of the
// group's earlier words + the bits below c in its word
__device__ __forceinline__ int bm_rank(const u64 *bm, const u16 *g4, const int *blk, long long c) {
    const int w = (int)(c >> 6), gi = w >> 2, sub = w & 3;
    const ulonglong2 lo = reinterpret_cast<const ulonglong2 *>(bm)[gi * 2];
    const ulonglong2 hi = reinterpret_cast<const ulonglong2 *>(bm)[gi * 2 + 1];
    const u64 word = sub == 0 ? lo.x : sub == 1 ? lo.y : sub == 2 ? hi.x : hi.y;
    int rk = blk[w / RH_BLK] + g4[gi] + __popcll(word & ((1ull << (c & 63)) - 1ull));
    rk += sub > 0 ? __popcll(lo.x) : 0;
    rk += sub > 1 ? __popcll(lo.y) : 0;
    rk += sub > 2 ? __popcll(hi.x) : 0;
    return rk;
}

__global__ __launch_bounds__(RH_NT) void k_rows_bitmap(RowsArgs g, int *Tc, double *Tx, int *Tr,
                                                      unsigned long long *tcur) {
    {  // (hub rows, past kRowsHubProducts: the windowed or the DR kernels')
        const int4 le0 = g.list[blockIdx.x];
        if (g.E[le0.y + le0.z] - g.E[le0.y] > kRowsHubProducts) return;  // (workgroup-uniform)
    }
    __shared__ __align__(16) u64 bm[RH_WORDS];
    __shared__ u16 g4[RH_NGRP];       // each 4-word group's bits before it in its block
    __shared__ int blk[RH_NBLK];      // each block's bits before it in the window
    __shared__ WalkTab wt;
    __shared__ int red[3 * (RH_NT / 64)];
    constexpr int NW = RH_NT / 64;
    RP_INIT
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int4 le = g.list[blockIdx.x];
    const int r = le.x, a0 = le.y, k = le.z;
    const long long base = g.E[a0];
    // (rows of more runs or a wider span: the windowed kernels, k_rows_w*)
    if (k > OW_RUNS) return;  // (workgroup-uniform)
    const int P = (int)(g.E[a0 + k] - base);  // (<= kRowsHubProducts: hub rows left above)
    // run table (2 runs per thread; the walk table's LDS): product prefix, B
    // start -- and from the same loads the row's columns [lo, hi]
    int *const opre = reinterpret_cast<int *>(&wt);
    int *const obs = opre + OW_RUNS;
    int lo = INT_MAX, hi = -1;
    {
        int2 be0 = make_int2(0, 0), be1 = make_int2(0, 0);
        if (2 * tid < k) be0 = g.ebnd[a0 + 2 * tid];
        if (2 * tid + 1 < k) be1 = g.ebnd[a0 + 2 * tid + 1];
        const int l0 = be0.y - be0.x, l1 = be1.y - be1.x;
        const int f0 = l0 > 0 ? g.Bcol[be0.x] : INT_MAX, e0 = l0 > 0 ? g.Bcol[be0.y - 1] : -1;
        const int f1 = l1 > 0 ? g.Bcol[be1.x] : INT_MAX, e1 = l1 > 0 ? g.Bcol[be1.y - 1] : -1;
        const int inc = wave_incl_scan_dpp(l0 + l1);
        lo = wave_last(wave_incl_dpp(min(f0, f1), INT_MAX, OpMin{}));
        hi = wave_last(wave_incl_dpp(max(e0, e1), INT_MIN, OpMax{}));
        if (lane == 63) red[wv] = inc;
        if (lane == 0) {
            red[NW + wv] = lo;
            red[2 * NW + wv] = hi;
        }
        __syncthreads();
        int woff = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            woff += w < wv ? red[w] : 0;
            lo = min(lo, red[NW + w]);
            hi = max(hi, red[2 * NW + w]);
        }
        const int ex = woff + inc - l0 - l1;
        opre[2 * tid] = ex;
        opre[2 * tid + 1] = ex + l0;
        obs[2 * tid] = be0.x;
        obs[2 * tid + 1] = be1.x;
    }
    if ((long long)hi - lo >= RH_SPAN) return;  // (workgroup-uniform)
    {
        // one window, ONE walk: each product's column and value gathered together
        // once -- the first OW_CH products held in registers, the rest (rows past
        // OW_CH products) in this row's scratch slots -- then ranks; the bitmap's
        // LDS then holds the columns at their ranks (copied out coalesced) and
        // the values (ds_add_f64 at the ranks, copied out), OW_CV / OW_CH ranks
        // per pass.  No global atomic, no second walk over B.
        __shared__ long long s_toff;
        if (tid == 0 && P > OW_CH) s_toff = (long long)atomicAdd(tcur, (unsigned long long)(P - OW_CH));
        const int nwd = (int)(((long long)hi - lo + 64) >> 6);
        for (int i = tid; i < nwd; i += RH_NT) bm[i] = 0ull;
        __syncthreads();
        // products q = j * RH_NT + tid, four at a time: run search, then the
        // column, value and A value loads together
        auto gather4 = [&](int j0, int (&c4)[4], double (&x4)[4]) {
            int b[4], len2[4], q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                q[u] = (j0 + u) * RH_NT + tid;
                b[u] = 0;
                len2[u] = q[u] < P ? k : 0;
                c4[u] = -1;
                x4[u] = 0.0;
            }
            const bool ub[4] = {true, true, true, true};
            search_ilp(opre, b, len2, q, ub);  // b - 1 = the run holding product q
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (q[u] < P) {
                    const int jr = b[u] - 1;
                    const int pp = obs[jr] + q[u] - opre[jr];
                    c4[u] = g.Bcol[pp] - lo;
                    x4[u] = g.vA[a0 + jr] * g.Bval[pp];
                }
        };
        // the first RH_PPT products per thread: every run search first (LDS
        // only), then all their loads in flight together -- one memory round
        // trip for the register share instead of one per group of four (the
        // walk was 20 of a class-H row's 27 us on webbase)
        int cc[RH_PPT];
        double xx[RH_PPT];
        {
            int pa[RH_PPT], jr[RH_PPT];
#pragma unroll
            for (int j0 = 0; j0 < RH_PPT; j0 += 4) {
                int b[4], len2[4], q[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    q[u] = (j0 + u) * RH_NT + tid;
                    b[u] = 0;
                    len2[u] = q[u] < P ? k : 0;
                }
                const bool ub[4] = {true, true, true, true};
                if (j0 * RH_NT < P) search_ilp(opre, b, len2, q, ub);  // (workgroup-uniform)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    jr[j0 + u] = q[u] < P ? b[u] - 1 : -1;
                    pa[j0 + u] = q[u] < P ? obs[b[u] - 1] + q[u] - opre[b[u] - 1] : 0;
                }
            }
            double bv[RH_PPT], av[RH_PPT];
#pragma unroll
            for (int j = 0; j < RH_PPT; ++j) {
                cc[j] = jr[j] >= 0 ? g.Bcol[pa[j]] - lo : -1;
                bv[j] = jr[j] >= 0 ? g.Bval[pa[j]] : 0.0;
                av[j] = jr[j] >= 0 ? g.vA[a0 + jr[j]] : 0.0;
            }
#pragma unroll
            for (int j = 0; j < RH_PPT; ++j) xx[j] = av[j] * bv[j];
        }
#pragma unroll
        for (int j = 0; j < RH_PPT; ++j)
            if (cc[j] >= 0) atomicOr(&bm[cc[j] >> 6], 1ull << (cc[j] & 63));
        const long long toff = P > OW_CH ? s_toff - OW_CH : 0;  // scratch slot of product q: toff + q
        for (int j0 = RH_PPT; j0 * RH_NT < P; j0 += 4) {  // (workgroup-uniform) products past OW_CH
            int c4[4];
            double x4[4];
            gather4(j0, c4, x4);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (c4[u] >= 0) {
                    atomicOr(&bm[c4[u] >> 6], 1ull << (c4[u] & 63));
                    const long long t = toff + (j0 + u) * RH_NT + tid;
                    Tc[t] = c4[u];
                    Tx[t] = x4[u];
                }
        }
        __syncthreads();
        for (int b = wv; b < RH_NBLK; b += NW) {
            const int w0 = b * RH_BLK + lane * 8;
            int s0 = 0, s1 = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s0 += w0 + u < nwd ? __popcll(bm[w0 + u]) : 0;
                s1 += w0 + 4 + u < nwd ? __popcll(bm[w0 + 4 + u]) : 0;
            }
            const int inc = wave_incl_scan_dpp(s0 + s1);
            g4[w0 / 4] = (u16)(inc - s0 - s1);
            g4[w0 / 4 + 1] = (u16)(inc - s1);
            if (lane == 63) blk[b] = inc;
        }
        __syncthreads();
        if (wv == 0) {
            const int v = lane < RH_NBLK ? blk[lane] : 0;
            const int inc = wave_incl_scan_dpp(v);
            if (lane < RH_NBLK) blk[lane] = inc - v;
            if (lane == 63) red[0] = inc;
        }
        __syncthreads();
        const int wn = red[0];
        RP(6);
        int rk[RH_PPT];
#pragma unroll
        for (int j = 0; j < RH_PPT; ++j) rk[j] = cc[j] >= 0 ? bm_rank(bm, g4, blk, cc[j]) : 0;
        for (int q = OW_CH + tid; q < P; q += RH_NT) Tr[toff + q] = bm_rank(bm, g4, blk, Tc[toff + q]);
        RP(8);
        __syncthreads();  // (every bitmap read done: its LDS becomes the columns, then the values)
        RP(9);
        // the columns at their ranks in LDS (a column's products store the same
        // one), then out coalesced; OW_CV ranks per pass
        int *const cl = reinterpret_cast<int *>(bm);
        for (int r0 = 0; r0 < wn; r0 += OW_CV) {
#pragma unroll
            for (int j = 0; j < RH_PPT; ++j)
                if (cc[j] >= 0 && (unsigned)(rk[j] - r0) < (unsigned)OW_CV) cl[rk[j] - r0] = cc[j];
            for (int q = OW_CH + tid; q < P; q += RH_NT) {
                const int rq = Tr[toff + q] - r0;
                if ((unsigned)rq < (unsigned)OW_CV) cl[rq] = Tc[toff + q];
            }
            __syncthreads();
            const int n = min(OW_CV, wn - r0);
            for (int i = tid; i < n; i += RH_NT) g.Scol[base + r0 + i] = lo + cl[i];
            __syncthreads();
        }
        // the values: OW_CH ranks per pass
        double *const val = reinterpret_cast<double *>(bm);
        for (int r0 = 0; r0 < wn; r0 += OW_CH) {
            const int n = min(OW_CH, wn - r0);
            for (int i = tid; i < n; i += RH_NT) val[i] = 0.0;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < RH_PPT; ++j)
                if (cc[j] >= 0 && (unsigned)(rk[j] - r0) < (unsigned)OW_CH) atomicAdd(&val[rk[j] - r0], xx[j]);
            for (int q = OW_CH + tid; q < P; q += RH_NT) {
                const int rq = Tr[toff + q] - r0;
                if ((unsigned)rq < (unsigned)OW_CH) atomicAdd(&val[rq], Tx[toff + q]);
            }
            __syncthreads();
            RP(10);
            for (int i = tid; i < n; i += RH_NT) g.Sval[base + r0 + i] = val[i];
            __syncthreads();
        }
        if (tid == 0) g.rnnz[r] = wn;
        RP(7);
        RP_DONE(0);
        return;
    }
}

// the longest run of a row (entries a0 .. a0+k, products from the prefix E)
// and its entry (the first such), over the workgroup; red: 2 * (blockDim / 64) ints
__device__ __forceinline__ long long row_longest_run(const long long *E, int a0, int k, int *jl, int *red) {
    const int nw = blockDim.x >> 6, lane = lane_id(), wv = wave_id();
    long long best = -1;
    int bj = INT_MAX;
    for (int j0 = threadIdx.x; j0 < k; j0 += 4 * blockDim.x) {  // (four runs' loads in flight)
        long long e0[4], e1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = min(j0 + u * (int)blockDim.x, k - 1);
            e0[u] = E[a0 + j];
            e1[u] = E[a0 + j + 1];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (j0 + u * (int)blockDim.x < k && e1[u] - e0[u] > best) {
                best = e1[u] - e0[u];
                bj = j0 + u * (int)blockDim.x;
            }
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        const long long ob = __shfl_xor(best, d, 64);
        const int oj = __shfl_xor(bj, d, 64);
        if (ob > best || (ob == best && oj < bj)) {
            best = ob;
            bj = oj;
        }
    }
    __syncthreads();  // (red may hold an earlier phase's values)
    if (lane == 0) {
        red[2 * wv] = (int)min(best, (long long)INT_MAX);  // (a run is one B row: < 2^31)
        red[2 * wv + 1] = bj;
    }
    __syncthreads();
    best = -1;
    bj = INT_MAX;
    for (int w = 0; w < nw; ++w) {
        const long long ob = red[2 * w];
        const int oj = red[2 * w + 1];
        if (ob > best || (ob == best && oj < bj)) {
            best = ob;
            bj = oj;
        }
    }
    __syncthreads();
    *jl = bj;
    return best;
}

// ---- windowed rows (W rows): class-H rows that neither the one-walk bitmap
// kernel (more than OW_RUNS runs or a span past RH_SPAN) nor the dominant-run
// kernels take -- R-MAT hub rows (LiveJournal: rows of 10^5..10^7 products over
// 4 M columns, half of them repeated columns).  Each such row is cut into
// windows of 2^wb columns (wb per row, so that a window holds about W_UNIT
// products); a (row, window) pair is a UNIT, and units, not rows, are what the
// kernels spread over the GPU:
//   k_rows_wplan   a workgroup per class-H row: DR / one-walk / W, the W row's
//                  span, wb, its units and its chunks (W_CH products of one run
//                  batch each);
//   k_rows_wchunks the chunk list and each unit's row;
//   k_rows_wcount  a workgroup per chunk: the chunk's products counted per
//                  window in LDS, one global add per nonempty window;
//   k_rows_wscan   per W row, the units' counts scanned (bucket offsets inside
//                  the row's staging slots, later the output offsets);
//                  (that add's result: the chunk's place in the window's bucket);
//   k_rows_wscatter a workgroup per chunk: each product's (column, a*b) to its
//                  window's bucket in the row's staging, at the chunk's place
//                  plus an LDS cursor;
//   k_rows_wunit<0> a workgroup per unit: the bucket's columns ORed into an
//                  LDS bitmap of the window; its popcount is the unit's nnz;
//   k_rows_wunit<1> after the row scan (every count known): the bitmap again,
//                  ranks by popcount prefixes, the values added at their ranks
//                  in LDS, the unit's nonzeros straight into C in column order
//                  at the row's pointer + the unit's offset.  (Until round 6
//                  one unit kernel wrote them to an output area that a gather
//                  then copied into C, 24 B per nonzero; the split reads the
//                  bucket's columns twice, 4 B per product: a 60,000-row
//                  LiveJournal block 29.6 -> 29.2 ms.  Storing the count
//                  kernel's bitmaps for the fill to load, 2^wb bits per unit,
//                  measured 31.1 ms.)
//   k_rows_wsort   on the checked-scan path (list sizes read back with nnz(C)),
//                  units of at most WS_CAP products instead: a sort, no bitmap.
// Every product is read from B once for its column (counts) and once with its
// value (scatter), then through its bucket once; no global atomic per
// product, and a hub row's work is spread over as many workgroups as it has
// chunks and units.
constexpr int W_NT = RH_NT;        // (the run-batch tables are RH_NT wide)
constexpr int W_UNIT = 8192;       // products per unit, the target of wb
constexpr int W_MAXW = 8192;       // windows per row
constexpr int W_WBMIN = 8, W_WBMAX = 18;
constexpr int W_WORDS = (1 << W_WBMAX) / 64;  // bitmap words of the widest window: 32 KB
constexpr int W_BLK = 512;                    // words per rank block
constexpr int W_NBLK = W_WORDS / W_BLK;
constexpr int W_VCAP = 4096;                  // a unit's values per LDS pass
constexpr int W_RPT = 8;                      // a unit's products per thread held in registers
constexpr int WU_NT = 1024;                   // the unit fill's workgroup (W_RPT * WU_NT >= W_UNIT)
constexpr int WU_NT0 = 512;                   // the unit count's (its LDS: the bitmap alone)
constexpr int WS_NT = 256, WS_CAP = 4 * WS_NT;  // units of at most WS_CAP products: the sort fill
constexpr int WS_MAX = WS_CAP;                   // (the sort fill's units: 1 .. WS_MAX products)
constexpr int W_SPANK = 8192;                 // plan: rows past so many runs span all of B's columns

__device__ __forceinline__ int ceil_log2_ll(long long v) {
    int l = 0;
    while ((1ll << l) < v) ++l;
    return l;
}

// (W_NT threads) workgroup sum of a long long
__device__ __forceinline__ long long w_block_sum(long long x, long long *red) {
    constexpr int NW = W_NT / 64;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
    __syncthreads();
    if (lane_id() == 0) red[wave_id()] = x;
    __syncthreads();
    long long t = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += red[w];
    return t;
}

// a workgroup per class-H row i.  Outputs (zero unless a W row): wnw[i] units,
// wnch[i] chunks, wlo[i] first column, wwb[i] window bits;
// wst[0] += W rows' products, wst[1] / wst[2] += DR rows' products / rows.
__global__ __launch_bounds__(W_NT) void k_rows_wplan(RowsArgs g, int bn, long long unit, int *wnw, int *wnch,
                                                    int *wlo, int *wwb, long long *wmat,
                                                    unsigned long long *wst, long long *soff) {
    constexpr int NW = W_NT / 64;
    __shared__ int red[2 * NW];
    __shared__ long long red64[NW];
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int i = blockIdx.x;
    const int4 le = g.list[i];
    const int a0 = le.y, k = le.z;
    const long long base = g.E[a0], P = g.E[a0 + k] - base;
    int nw = 0, nch = 0, lo = 0, wb = 0;
    long long pw = 0;
    bool dr = false;
    if (P > kRowsHubProducts) {
        int jl;
        const long long L = row_longest_run(g.E, a0, k, &jl, red);
        dr = P - L <= DR_SMAX;
    }
    if (!dr) {
        // the span from the runs' first and last columns; rows past W_SPANK runs
        // (windowed anyway) take all of B's columns instead of that walk
        int l = k > W_SPANK ? 0 : INT_MAX, h = k > W_SPANK ? bn - 1 : -1;
        for (int j0 = tid; j0 < (k > W_SPANK ? 0 : k); j0 += 4 * W_NT) {  // (four runs' loads in flight)
            int2 be[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) be[u] = j0 + u * W_NT < k ? g.ebnd[a0 + j0 + u * W_NT] : make_int2(0, 0);
            int cl[4], ch[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                cl[u] = be[u].y > be[u].x ? g.Bcol[be[u].x] : INT_MAX;
                ch[u] = be[u].y > be[u].x ? g.Bcol[be[u].y - 1] : -1;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                l = min(l, cl[u]);
                h = max(h, ch[u]);
            }
        }
        l = wave_last(wave_incl_dpp(l, INT_MAX, OpMin{}));
        h = wave_last(wave_incl_dpp(h, INT_MIN, OpMax{}));
        __syncthreads();
        if (lane == 0) {
            red[wv] = l;
            red[NW + wv] = h;
        }
        __syncthreads();
        l = red[0];
        h = red[NW];
#pragma unroll
        for (int w = 1; w < NW; ++w) {
            l = min(l, red[w]);
            h = max(h, red[NW + w]);
        }
        // (the one-walk bitmap kernel's rows: k_rows_bitmap's own test)
        const bool onewalk = P <= kRowsHubProducts && k <= OW_RUNS && (long long)h - l < RH_SPAN;
        if (!onewalk && P > 0) {
            const long long span = (long long)h - l + 1;
            const int lg = ceil_log2_ll(span);
            wb = ceil_log2_ll((span * unit + P - 1) / P);
            wb = max(wb, lg - 13);                // (at most W_MAXW windows)
            wb = max(wb, min(lg - 10, W_WBMAX));  // (at most 1,024 windows where the widest window allows)
            wb = min(max(wb, W_WBMIN), W_WBMAX);
            nw = (int)((span + (1ll << wb) - 1) >> wb);
            lo = l;
            pw = P;
            // chunks: per run batch of RH_NT runs, W_CH products each
            long long c = 0;
            for (int b0 = tid * RH_NT; b0 < k; b0 += W_NT * RH_NT) {
                const long long tot = g.E[a0 + min(k, b0 + RH_NT)] - g.E[a0 + b0];
                c += (tot + W_CH - 1) / W_CH;
            }
            nch = (int)w_block_sum(c, red64);
        }
    }
    if (tid == 0) {
        wnw[i] = nw;
        wnch[i] = nch;
        wlo[i] = lo;
        wwb[i] = wb;
        wmat[i] = (long long)nch * nw;
        if (nw) soff[le.x] = -1;  // (the compaction skips the row: k_rows_wunit<1> writes it)
        if (pw) atomicAdd(&wst[0], (unsigned long long)pw);
        if (dr) {
            atomicAdd(&wst[1], (unsigned long long)P);
            atomicAdd(&wst[2], 1ull);
        }
    }
}

// a workgroup per class-H row i: its units' row (umap) and its chunks
// (class-H index, batch, slice) from cbase[i], each chunk's row of the
// per-window offset matrix at cmoff (wnw, wnch, wmat scanned: ubase, cbase, mbase)
__global__ __launch_bounds__(WG) void k_rows_wchunks(RowsArgs g, const int *ubase, const int *cbase,
                                                    const long long *mbase, int4 *chunks, long long *cmoff,
                                                    int *umap) {
    __shared__ int red[WAVES];
    const int i = blockIdx.x;
    const int u0 = ubase[i], nw = ubase[i + 1] - u0;
    if (nw == 0) return;  // (workgroup-uniform)
    for (int w = threadIdx.x; w < nw; w += WG) umap[u0 + w] = i;
    const int4 le = g.list[i];
    const int a0 = le.y, k = le.z, c0 = cbase[i];
    const long long m0 = mbase[i];
    int carry = 0;
    for (int bb = 0; bb * RH_NT < k; bb += WG) {  // (workgroup-uniform) WG batches at a time
        const int b = bb + threadIdx.x;
        int ns = 0;
        if (b * RH_NT < k) {
            const long long tot = g.E[a0 + min(k, (b + 1) * RH_NT)] - g.E[a0 + b * RH_NT];
            ns = (int)((tot + W_CH - 1) / W_CH);
        }
        int tot = 0;
        const int off = carry + block_excl_scan(ns, &tot, red);
        for (int j = 0; j < ns; ++j) {
            const int c = c0 + off + j;
            chunks[c] = make_int4(i, b, j, 0);
            cmoff[c] = m0 + (long long)(off + j) * nw;
        }
        carry += tot;
    }
}

// lanes of a wave holding consecutive products: runs of equal window w
// (w = -1 for invalid lanes, a suffix).  Returns the boundary mask (a bit per
// lane that starts a run); *len = the run's length for its first lane.
__device__ __forceinline__ u64 wave_runs(int w, int *len) {
    const int lane = lane_id();
    const int wp = __shfl_up(w, 1, 64);
    const u64 bm = __ballot(lane == 0 || wp != w);
    const u64 above = bm & ~((2ull << lane) - 1ull);  // (lane 63: none)
    *len = (above ? __builtin_ctzll(above) : 64) - lane;
    return bm;
}

// the chunk's products counted per window into LDS hist (zeroed by the caller
// before; the batch's run table loaded into wt); returns the row's window shape
__device__ __forceinline__ void w_chunk_hist(const RowsArgs &g, int4 ch, int lo, int wb, int *hist, WalkTab &wt,
                                             unsigned short *rmap, int *red) {
    const int4 le = g.list[ch.x];
    const int a0 = le.y, k = le.z, b0 = ch.y * RH_NT;
    rows_batch(g, a0, k, b0, wt);  // (its barriers also order the caller's zeroing)
    const int q0 = ch.z * W_CH, q1 = min(wt.tot, q0 + W_CH);
    // one LDS add per run of equal windows in a wave (the runs of B are
    // column-sorted: neighbouring lanes mostly share a window)
    batch_walk<false>(g, min(RH_NT, k - b0), q0, q1, wt, [&](int c, double, bool v) {
        const int w = v ? (c - lo) >> wb : -1;
        int len;
        const u64 bm = wave_runs(w, &len);
        if (v && (bm >> lane_id() & 1ull)) atomicAdd(&hist[w], len);
    }, rmap, red);
    __syncthreads();
}

__global__ __launch_bounds__(W_NT) void k_rows_wcount(RowsArgs g, const int4 *chunks, const long long *cmoff,
                                                     const int *wlo, const int *wwb, const int *ubase, int *ucnt,
                                                     int *cbo) {
    __shared__ int hist[W_MAXW];
    __shared__ WalkTab wt;
    __shared__ __align__(16) unsigned short rmap[8 * RH_NT];  // (two maps: batch_walk)
    __shared__ int red[RH_NT / 64];
    const int4 ch = chunks[blockIdx.x];
    const int u0 = ubase[ch.x], nw = ubase[ch.x + 1] - u0;
    for (int w = threadIdx.x; w < nw; w += W_NT) hist[w] = 0;
    w_chunk_hist(g, ch, wlo[ch.x], wwb[ch.x], hist, wt, rmap, red);
    int *const cb = cbo + cmoff[blockIdx.x];  // the chunk's place in each window's bucket
    for (int w = threadIdx.x; w < nw; w += W_NT)
        if (hist[w]) cb[w] = atomicAdd(&ucnt[u0 + w], hist[w]);
}

// a unit's work record (k_rows_wscan writes it beside the bucket offsets): the
// unit kernel's one dependent load before its bucket loads (reading umap ->
// list -> E first cost three round trips per unit)
struct WUnit {
    long long s0;   // its bucket in the row's staging slots
    int wlo0;       // its window's first column
    int wb;         // window bits
    int n;          // its bucket's products
    int row;        // its C row
};

// per W row (a workgroup per class-H row): out[u] = exclusive scan of in[u]
// over the row's units; rnnz (optional) gets the row's total; rec (optional,
// with wlo, wwb) the units' work records, and the fill lists: units of 1 ..
// WS_CAP products appended to ulist (*lcnt64 bits 0..20: the sort fill's); for
// the bitmap fill, units past W_RPT * WU_NT products to the back of ulist2,
// ulist2[nu - 1 - i] (bits 21..41), the others to its front (bits 42..62) -- the
// longest units dispatched first, so that none starts at the fill's end
__global__ __launch_bounds__(W_NT) void k_rows_wscan(RowsArgs g, const int *ubase, const int *in, int *out,
                                                    int *rnnz, WUnit *rec = nullptr, const int *wlo = nullptr,
                                                    const int *wwb = nullptr, int *ulist = nullptr,
                                                    int *ulist2 = nullptr, unsigned long long *lcnt64 = nullptr,
                                                    int nu = 0) {
    constexpr int NW = W_NT / 64, PT = W_MAXW / W_NT;
    __shared__ int red[NW];
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int u0 = ubase[blockIdx.x], nw = ubase[blockIdx.x + 1] - u0;
    if (nw == 0) return;  // (workgroup-uniform)
    int v[PT], sum = 0;
#pragma unroll
    for (int t = 0; t < PT; ++t) {
        const int w = tid * PT + t;
        v[t] = w < nw ? in[u0 + w] : 0;
        sum += v[t];
    }
    const int inc = wave_incl_scan_dpp(sum);
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    int off = inc - sum, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        off += w < wv ? red[w] : 0;
        tot += red[w];
    }
    long long rb = 0;
    int lo = 0, wb = 0, row = 0;
    if (rec) {  // (kernel-uniform)
        const int4 le = g.list[blockIdx.x];
        rb = g.E[le.y];
        row = le.x;
        lo = wlo[blockIdx.x];
        wb = wwb[blockIdx.x];
    }
#pragma unroll
    for (int t = 0; t < PT; ++t) {
        const int w = tid * PT + t;
        if (w < nw) {
            out[u0 + w] = off;
            if (rec) rec[u0 + w] = WUnit{rb + off, lo + (w << wb), wb, v[t], row};
        }
        off += v[t];
    }
    if (rnnz && tid == 0) rnnz[g.list[blockIdx.x].x] = tot;
    if (ulist) {  // (kernel-uniform) the fill lists, one atomic per wave and list
        constexpr int HEAVY = W_RPT * WU_NT;
        int ns = 0, nh = 0, nm = 0;
#pragma unroll
        for (int t = 0; t < PT; ++t) {
            ns += v[t] > 0 && v[t] <= WS_MAX;
            nh += v[t] > HEAVY;
            nm += v[t] > WS_MAX && v[t] <= HEAVY;
        }
        const int is = wave_incl_scan_dpp(ns), ih = wave_incl_scan_dpp(nh), im = wave_incl_scan_dpp(nm);
        // one atomic per wave for the three lists: 21-bit fields of a u64 (nu < 2^21,
        // the host's condition); three same-address atomics per wave cost ~0.17 ms
        // per LiveJournal block
        unsigned long long old = 0;
        if (lane == 63 && (is | ih | im))
            old = atomicAdd(lcnt64, (unsigned long long)is | ((unsigned long long)ih << 21) |
                                        ((unsigned long long)im << 42));
        old = ((unsigned long long)__shfl((int)(old >> 32), 63, 64) << 32) | (u32)__shfl((int)old, 63, 64);
        int ps = (int)(old & 0x1fffff) + is - ns, ph = (int)((old >> 21) & 0x1fffff) + ih - nh,
            pm = (int)(old >> 42) + im - nm;
#pragma unroll
        for (int t = 0; t < PT; ++t) {
            const int w = tid * PT + t;
            if (v[t] > 0 && v[t] <= WS_MAX) ulist[ps++] = u0 + w;
            else if (v[t] > HEAVY) ulist2[nu - 1 - ph++] = u0 + w;
            else if (v[t] > WS_MAX) ulist2[pm++] = u0 + w;
        }
    }
}

// the chunk's products to their windows' buckets in the row's staging slots
// (bucket u at E[a0] + ubo[u]; the chunk's place in it from k_rows_wcount).
// Each product is stored at its window's LDS cursor.  (Binning each sub-batch
// by window in LDS first, then writing it out in window order, measured no
// faster on the LiveJournal block: 2.744 vs 2.746 ms; removed.)
__global__ __launch_bounds__(W_NT) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_rows_wscatter(RowsArgs g, const int4 *chunks, const long long *cmoff,
                                                       const int *wlo, const int *wwb, const int *ubase,
                                                       const int *ubo, const int *cbo) {
    // cursors of up to W_MAXW windows, the run map above them
    __shared__ __align__(16) unsigned char lds[W_MAXW * 4 + 8 * RH_NT * 2];  // (two run maps: batch_walk)
    __shared__ WalkTab wt;
    __shared__ int red[W_NT / 64];
    int *const cur = reinterpret_cast<int *>(lds);  // row-relative slots (windows not reached: unused)
    unsigned short *const rm = reinterpret_cast<unsigned short *>(lds + W_MAXW * 4);
    const int tid = threadIdx.x;
    const int4 ch = chunks[blockIdx.x];
    const int u0 = ubase[ch.x], nw = ubase[ch.x + 1] - u0;
    const int lo = wlo[ch.x], wb = wwb[ch.x];
    const int *const cb = cbo + cmoff[blockIdx.x];
    for (int w = tid; w < nw; w += W_NT) cur[w] = ubo[u0 + w] + cb[w];
    const int4 le = g.list[ch.x];
    const int a0 = le.y, k = le.z, b0 = ch.y * RH_NT;
    rows_batch(g, a0, k, b0, wt);  // (its barriers also order the cursors above)
    const long long base = g.E[a0];
    const int q0 = ch.z * W_CH, q1 = min(wt.tot, q0 + W_CH), nb = min(RH_NT, k - b0);
    // a run of equal windows in a wave takes its slots with one LDS add (its
    // first lane's), so neighbouring lanes store to neighbouring slots
    batch_walk<true>(g, nb, q0, q1, wt, [&](int c, double x, bool v) {
        const int lane = lane_id();
        const int w = v ? (c - lo) >> wb : -1;
        int len;
        const u64 bm = wave_runs(w, &len);
        int b = 0;
        if (v && (bm >> lane & 1ull)) b = atomicAdd(&cur[w], len);
        const int hl = 63 - __builtin_clzll(bm & ((2ull << lane) - 1ull));  // this lane's run start
        const int hb = __shfl(b, hl, 64);
        if (v) {
            const long long o = base + hb + (lane - hl);
            g.Scol[o] = c;
            g.Sval[o] = x;
        }
    }, rm, red);
}

// rank of column c inside a unit's window (bitmap bm, block and group prefixes)
__device__ __forceinline__ int w_rank(const u64 *bm, const u16 *g4, const int *blk, int c) {
    const int w = c >> 6, gi = w >> 2, sub = w & 3;
    const ulonglong2 lo = reinterpret_cast<const ulonglong2 *>(bm)[gi * 2];
    const ulonglong2 hi = reinterpret_cast<const ulonglong2 *>(bm)[gi * 2 + 1];
    const u64 word = sub == 0 ? lo.x : sub == 1 ? lo.y : sub == 2 ? hi.x : hi.y;
    int rk = blk[w / W_BLK] + g4[gi] + __popcll(word & ((1ull << (c & 63)) - 1ull));
    rk += sub > 0 ? __popcll(lo.x) : 0;
    rk += sub > 1 ? __popcll(lo.y) : 0;
    rk += sub > 2 ? __popcll(hi.x) : 0;
    return rk;
}

// a workgroup per unit u (its record R: bucket of R.n products at R.s0, window
// of 2^R.wb columns from R.wlo0, C row R.row).
//   MODE 0 (count): the bucket's columns ORed into an LDS bitmap of the window;
//     ucount[u] = its popcount.
//   MODE 1 (fill, after the row scan): the bitmap again, ranks by popcount
//     prefixes (u16 per 4-word group, int per 512-word block), the values added
//     at their ranks in LDS, the unit's nonzeros written in column order into C
//     at Crp[R.row] + uoff[u].
template <int MODE, int NT>
__global__ __launch_bounds__(NT) void k_rows_wunit(RowsArgs g, const WUnit *urec, int *ucount, const int *uoff,
                                                    const int *Crp, int *Ccol, double *Cval,
                                                    const int *ulist = nullptr, int ulast = 0,
                                                    int nheavy = 0) {
    constexpr int NW = NT / 64;
    __shared__ __align__(16) u64 bm[W_WORDS];
    __shared__ u16 g4[W_WORDS / 4];
    __shared__ int blk[W_NBLK];
    __shared__ __align__(16) double vals[W_VCAP];
    __shared__ int red[NW];
    RP_INIT
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int b = blockIdx.x;  // (with a list: its heavy units from the back first, then the rest from the front)
    const int u = ulist ? ulist[b < nheavy ? ulast - b : b - nheavy] : b;
    const WUnit R = urec[u];
    const int n = R.n;
    if (n == 0) {  // (workgroup-uniform)
        if (MODE == 0 && tid == 0) ucount[u] = 0;
        return;
    }
    const int wb = R.wb;
    const long long wlo0 = R.wlo0;
    const long long s0 = R.s0;
    const int nwd = 1 << (wb - 6);
    if constexpr (MODE == 0) {
        for (int w = tid; w < nwd; w += NT) bm[w] = 0ull;
        int cc[W_RPT];
#pragma unroll
        for (int t = 0; t < W_RPT; ++t) {
            const int q = t * NT + tid;
            cc[t] = q < n ? (int)(g.Scol[s0 + q] - wlo0) : -1;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < W_RPT; ++t)
            if (cc[t] >= 0) atomicOr(&bm[cc[t] >> 6], 1ull << (cc[t] & 63));
        for (int q = W_RPT * NT + tid; q < n; q += NT) {
            const int c = (int)(g.Scol[s0 + q] - wlo0);
            atomicOr(&bm[c >> 6], 1ull << (c & 63));
        }
        __syncthreads();
        int cnt = 0;
        for (int w = tid; w < nwd; w += NT) cnt += __popcll(bm[w]);
        cnt = wave_sum(cnt);
        if (lane == 0) red[wv] = cnt;
        __syncthreads();
        if (tid == 0) {
            int t = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) t += red[w];
            ucount[u] = t;
        }
        RP_DONE(0);
        return;
    }
    // (fill) the first W_RPT * NT products in registers (the rest read again
    // below), the bitmap again, the unit's place in C
    for (int w = tid; w < nwd; w += NT) bm[w] = 0ull;
    int cc[W_RPT];
    double xx[W_RPT];
#pragma unroll
    for (int t = 0; t < W_RPT; ++t) {
        const int q = t * NT + tid;
        cc[t] = q < n ? (int)(g.Scol[s0 + q] - wlo0) : -1;
        xx[t] = q < n ? g.Sval[s0 + q] : 0.0;
    }
    const long long o0 = (long long)Crp[R.row] + uoff[u];
    __syncthreads();
#pragma unroll
    for (int t = 0; t < W_RPT; ++t)
        if (cc[t] >= 0) atomicOr(&bm[cc[t] >> 6], 1ull << (cc[t] & 63));
    for (int q = W_RPT * NT + tid; q < n; q += NT) {
        const int c = (int)(g.Scol[s0 + q] - wlo0);
        atomicOr(&bm[c >> 6], 1ull << (c & 63));
    }
    __syncthreads();
    RP(1);
    // ranks: a wave per W_BLK-word block (a lane: two 4-word groups), then the blocks
    for (int bb = wv; bb * W_BLK < nwd; bb += NW) {
        const int w0 = bb * W_BLK + lane * 8;
        int t0 = 0, t1 = 0;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            t0 += w0 + v < nwd ? __popcll(bm[w0 + v]) : 0;
            t1 += w0 + 4 + v < nwd ? __popcll(bm[w0 + 4 + v]) : 0;
        }
        const int inc = wave_incl_scan_dpp(t0 + t1);
        if (w0 < nwd) g4[w0 / 4] = (u16)(inc - t0 - t1);
        if (w0 + 4 < nwd) g4[w0 / 4 + 1] = (u16)(inc - t1);
        if (lane == 63) blk[bb] = inc;
    }
    __syncthreads();
    const int nb = (nwd + W_BLK - 1) / W_BLK;
    if (wv == 0) {
        const int v = lane < nb ? blk[lane] : 0;
        const int inc = wave_incl_scan_dpp(v);
        if (lane < nb) blk[lane] = inc - v;
        if (lane == 63) red[0] = inc;
    }
    __syncthreads();
    const int wn = red[0];
    RP(2);
    int rk[W_RPT];
#pragma unroll
    for (int t = 0; t < W_RPT; ++t) rk[t] = cc[t] >= 0 ? w_rank(bm, g4, blk, cc[t]) : 0;
    static_assert(2 * W_WORDS >= W_RPT * NT, "the bitmap's LDS holds a column per rank (wn <= n)");
    if (n <= W_RPT * NT) {  // (workgroup-uniform) every product in registers
        // the bitmap is done with once the ranks are: its LDS takes each rank's
        // column (a column's products store the same one), the values are
        // summed at their ranks W_VCAP at a time, and both go out coalesced
        // (consecutive lanes, consecutive ranks) -- not a thread per bitmap
        // word emitting its bits
        int *const cl = reinterpret_cast<int *>(bm);
        __syncthreads();  // (every rank read from the bitmap)
#pragma unroll
        for (int t = 0; t < W_RPT; ++t)
            if (cc[t] >= 0) cl[rk[t]] = cc[t];
        RP(3);
        for (int r0 = 0; r0 < wn; r0 += W_VCAP) {  // (workgroup-uniform)
            const int r1 = min(wn, r0 + W_VCAP);
            for (int j = tid; j < r1 - r0; j += NT) vals[j] = 0.0;
            __syncthreads();
#pragma unroll
            for (int t = 0; t < W_RPT; ++t)
                if (cc[t] >= 0 && (unsigned)(rk[t] - r0) < (unsigned)W_VCAP) atomicAdd(&vals[rk[t] - r0], xx[t]);
            __syncthreads();
            RP(4);
            for (int j = tid; j < r1 - r0; j += NT) {
                Ccol[o0 + r0 + j] = (int)(wlo0 + cl[r0 + j]);
                Cval[o0 + r0 + j] = vals[j];
            }
            __syncthreads();  // (the pass's values read before the next pass zeroes them)
            RP(5);
        }
        RP_DONE(0);
        return;
    }
#ifdef TSG_ROWS_PROF
    for (int k = 0; k < 3; ++k) {  // (the large units' phases 0..2 as 6..8)
        rp_acc[6 + k] += rp_acc[k];
        rp_acc[k] = 0;
    }
#endif
    for (int r0 = 0; r0 < wn; r0 += W_VCAP) {  // (workgroup-uniform; one pass unless wn > W_VCAP)
        const int r1 = min(wn, r0 + W_VCAP);
        for (int j = tid; j < r1 - r0; j += NT) vals[j] = 0.0;
        __syncthreads();
#pragma unroll
        for (int t = 0; t < W_RPT; ++t)
            if (cc[t] >= 0 && (unsigned)(rk[t] - r0) < (unsigned)W_VCAP) atomicAdd(&vals[rk[t] - r0], xx[t]);
        for (int q = W_RPT * NT + tid; q < n; q += NT) {
            const int c = (int)(g.Scol[s0 + q] - wlo0);
            const int rq = w_rank(bm, g4, blk, c) - r0;
            if ((unsigned)rq < (unsigned)W_VCAP) atomicAdd(&vals[rq], g.Sval[s0 + q]);
        }
        __syncthreads();
        RP(9);
        // emit: a thread per bitmap word, its columns at their ranks
        for (int w = tid; w < nwd; w += NT) {
            u64 word = bm[w];
            if (!word) continue;
            int r = w_rank(bm, g4, blk, w * 64);
            if (r >= r1) continue;
            while (word) {
                const int bit = __builtin_ctzll(word);
                word &= word - 1ull;
                if (r >= r0 && r < r1) {
                    Ccol[o0 + r] = (int)(wlo0 + w * 64 + bit);
                    Cval[o0 + r] = vals[r - r0];
                }
                ++r;
            }
        }
        __syncthreads();  // (the pass's values read before the next pass zeroes them)
        RP(10);
    }
    RP(11);
    RP_DONE(0);
}

// a workgroup per unit of 1 .. WS_CAP products (the front of the fill list):
// the unit's nonzeros into C by a sort, not a window bitmap.  A sparse row's
// unit (LiveJournal: 2^18-column windows of ~600 products, nearly every column
// once) spent its time on the 32 KB bitmap's clear, sweeps and barriers at two
// workgroups per CU; here 16 KB of LDS, eight workgroups per CU.  Keys
// (column - wlo0) << 10 | position, unique: each wave sorts its 256 in
// registers, a bitonic merge over the waves' segments through LDS (only as
// many as the unit fills), then each run of equal columns is summed in
// position order by its first element and written at its rank.
__global__ __launch_bounds__(WS_NT) void k_rows_wsort(RowsArgs g, const WUnit *urec, const int *ulist,
                                                    const int *uoff, const int *Crp, int *Ccol, double *Cval) {
    constexpr int NW = WS_NT / 64, SEG = 256, IB = WS_CAP == 1024 ? 10 : WS_CAP == 2048 ? 11 : 12;
    static_assert((1 << IB) == WS_CAP && (W_WBMAX + IB) < 32, "keys: window column and position in a u32");
    __shared__ __align__(16) u32 kb[2][WS_CAP];
    __shared__ __align__(16) double V[WS_CAP];
    __shared__ int red[NW];
    const int u = ulist[blockIdx.x];
    const WUnit R = urec[u];
    const int n = R.n;  // (1 .. WS_CAP)
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int e0 = 4 * tid;  // (= 256 wv + 4 lane: a wave's segment of positions)
    u32 x[4];
    double xv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int q = e0 + k;
        x[k] = q < n ? ((u32)(g.Scol[R.s0 + q] - R.wlo0) << IB) | (u32)q : ~0u;
        xv[k] = q < n ? g.Sval[R.s0 + q] : 0.0;
    }
    const long long o0 = (long long)Crp[R.row] + uoff[u];
    int npow = SEG;  // the sort's length: n padded to a power of two (~0u keys)
    while (npow < n) npow <<= 1;
    const bool act = wv * SEG < npow;  // (wave-uniform)
    if (e0 < n) reinterpret_cast<double4 *>(V)[tid] = make_double4(xv[0], xv[1], xv[2], xv[3]);
    if (wv * SEG < n) wave_sort256(x, lane);
    if (act) *reinterpret_cast<uint4 *>(kb[0] + e0) = make_uint4(x[0], x[1], x[2], x[3]);
    __syncthreads();
    int src = 0;
    auto cmpx = [&](const uint4 y, bool rev, bool keep_min) {
        const u32 yy[4] = {rev ? y.w : y.x, rev ? y.z : y.y, rev ? y.y : y.z, rev ? y.x : y.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = keep_min ? min(x[k], yy[k]) : max(x[k], yy[k]);
    };
    for (int K = 2 * SEG; K <= npow; K <<= 1) {  // (workgroup-uniform)
        if (act) cmpx(*reinterpret_cast<const uint4 *>(kb[src] + (e0 ^ (K - 4))), true, (e0 & (K >> 1)) == 0);
        for (int J = K >> 2; J >= SEG; J >>= 1) {
            src ^= 1;
            if (act) *reinterpret_cast<uint4 *>(kb[src] + e0) = make_uint4(x[0], x[1], x[2], x[3]);
            __syncthreads();
            if (act) cmpx(*reinterpret_cast<const uint4 *>(kb[src] + (e0 ^ J)), false, (e0 & J) == 0);
        }
        if (act) bitonic_merge<256, 128>(x, lane);
        src ^= 1;
        if (act) *reinterpret_cast<uint4 *>(kb[src] + e0) = make_uint4(x[0], x[1], x[2], x[3]);
        __syncthreads();
    }
    const u32 *const ks = kb[src];  // the sorted keys (positions >= n: ~0u)
    // heads: the first position of each column; their ranks by a workgroup scan
    u32 prev = e0 > 0 && e0 - 1 < n ? ks[e0 - 1] >> IB : ~0u;
    bool hd[4];
    int nh = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const u32 col = x[k] >> IB;
        hd[k] = e0 + k < n && col != prev;
        prev = col;
        nh += hd[k];
    }
    const int inc = wave_incl_scan_dpp(nh);
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    int rk = inc - nh;
#pragma unroll
    for (int w = 0; w < NW; ++w) rk += w < wv ? red[w] : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (hd[k]) {
            const u32 col = x[k] >> IB;
            double sum = V[x[k] & (WS_CAP - 1)];
            for (int p = e0 + k + 1; p < n; ++p) {  // (the column's other products, in position order)
                const u32 y = ks[p];
                if ((y >> IB) != col) break;
                sum += V[y & (WS_CAP - 1)];
            }
            Ccol[o0 + rk] = (int)(R.wlo0 + (long long)col);
            Cval[o0 + rk] = sum;
            ++rk;
        }
}

// ---- hub rows dominated by one run (mawi: a hub neighbour's C row is the
// hub's whole B row plus a few entries): the row is the dominant run L with
// the other runs' products S (at most DR_SMAX) inserted.
//   k_rows_dr_prep, a workgroup per row: S expanded, sorted by (column,
//     position) in LDS and summed per column; each column's insertion point p
//     in L (binary search of the B row) and whether L holds the column (then
//     its sum joins that element); the row's nnz = |L| + the inserted columns;
//     the row's chunks of DR_CH elements of L enqueued.
//   k_rows_dr_fill (after the row scan: the prep's counts are exact), a
//     workgroup per chunk: L streamed (coalesced) straight into C at the
//     row's pointer + i + (inserted columns before it), the inserted
//     columns of its range beside them.  For L's element i the S columns
//     before it are those with p <= i that L does not hold; an S column goes
//     to p + (inserted columns before it).
struct DrRow {
    long long base;  // staging offset
    int r, bs, L, nu;
    double aL;
};
struct DrEnt {     // one S column (sorted by column): insertion point, kind, column, sum
    int p;           // first element of L at or past the column
    int nd;          // inserted (not in L) columns before this one in S
    int col;
    int dup;         // 1: L holds the column
    double val;
};
constexpr int DR_NT = 1024;

__global__ __launch_bounds__(DR_NT) void k_rows_dr_prep(RowsArgs g, long long *soff, DrRow *rows, DrEnt *ents,
                                                        int *ord, int4 *chunks, int *nchunk, int *ndr,
                                                        int enq) {
    constexpr int NW = DR_NT / 64;
    __shared__ unsigned long long sk[DR_SMAX];  // (column << 12 | S position), sorted
    __shared__ double sv[DR_SMAX];              // S values by S position
    __shared__ int red[2 * NW + 2];
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int4 le = g.list[blockIdx.x];
    const int r = le.x, a0 = le.y, k = le.z;
    const long long base = g.E[a0];
    const long long P = g.E[a0 + k] - base;
    if (P <= kRowsHubProducts) return;  // (workgroup-uniform)
    int jl;
    const long long L = row_longest_run(g.E, a0, k, &jl, red);
    const int nS = (int)(P - L);
    if (nS > DR_SMAX) return;  // (a windowed row)
    __shared__ int s_h;
    if (tid == 0) s_h = atomicAdd(ndr, 1);  // this row's slot among the DR rows
    const long long eL = g.E[a0 + jl] - base;  // L's first product in the row's product order
    const int2 bL = g.ebnd[a0 + jl];
    // S: the row's products outside L, in product order; position q -> the row's
    // product q' (q past L's start skips L), its entry by a binary search of E
    int npow = 1;
    while (npow < nS) npow <<= 1;
    for (int q = tid; q < npow; q += DR_NT) {
        if (q >= nS) {
            sk[q] = ~0ull;
            continue;
        }
        const long long qq = base + (q < eL ? q : q + L);
        int lo = a0, hi = a0 + k;  // the last entry a with E[a] <= qq
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (g.E[mid] <= qq) lo = mid; else hi = mid;
        }
        const int pb = g.ebnd[lo].x + (int)(qq - g.E[lo]);
        const int c = g.Bcol[pb];
        sv[q] = g.vA[lo] * g.Bval[pb];
        sk[q] = ((unsigned long long)(unsigned)c << 12) | (unsigned)q;
    }
    __syncthreads();
    // bitonic sort of npow keys in LDS
    for (int K = 2; K <= npow; K <<= 1)
        for (int J = K >> 1; J > 0; J >>= 1) {
            for (int i = tid; i < npow; i += DR_NT) {
                const int ij = i ^ J;
                if (ij > i) {
                    const unsigned long long a = sk[i], b = sk[ij];
                    const bool asc = (i & K) == 0;
                    if ((a > b) == asc) {
                        sk[i] = b;
                        sk[ij] = a;
                    }
                }
            }
            __syncthreads();
        }
    // per column (heads in sorted order): its sum in sorted order, insertion
    // point in L, whether L holds it
    int nh = 0;
    int hq[DR_SMAX / DR_NT];
#pragma unroll
    for (int u = 0; u < DR_SMAX / DR_NT; ++u) {
        const int t = tid * (DR_SMAX / DR_NT) + u;
        hq[u] = t < nS && (t == 0 || (sk[t] >> 12) != (sk[t - 1] >> 12));
        nh += hq[u];
    }
    const int inc = wave_incl_scan_dpp(nh);
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    int o = inc - nh, nu = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        o += w < wv ? red[w] : 0;
        nu += red[w];
    }
    const int h = s_h;  // (written before the barriers above)
    DrEnt *const E8 = ents + (long)h * DR_SMAX;
    const int oslot = o;  // this thread's first entry
    int ndp = 0;          // this thread's columns not in L
    int mydup[DR_SMAX / DR_NT];
#pragma unroll
    for (int u = 0; u < DR_SMAX / DR_NT; ++u) {
        const int t = tid * (DR_SMAX / DR_NT) + u;
        mydup[u] = 0;
        if (!hq[u]) continue;
        const int c = (int)(sk[t] >> 12);
        double sum = sv[sk[t] & 4095u];
        for (int j = t + 1; j < nS && (int)(sk[j] >> 12) == c; ++j) sum += sv[sk[j] & 4095u];  // (ascending)
        int lo = 0, hi = (int)L;  // first element of L at or past c
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (g.Bcol[bL.x + mid] < c) lo = mid + 1; else hi = mid;
        }
        mydup[u] = lo < L && g.Bcol[bL.x + lo] == c;
        ndp += !mydup[u];
        DrEnt e;
        e.p = lo;
        e.col = c;
        e.dup = mydup[u];
        e.val = sum;
        e.nd = 0;
        E8[o++] = e;
    }
    // inserted columns before each entry: exclusive scan of the not-in-L flags in S order
    __syncthreads();  // (red reused)
    const int inc2 = wave_incl_scan_dpp(ndp);
    if (lane == 63) red[wv] = inc2;
    __syncthreads();
    int nd = inc2 - ndp, ndt = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        nd += w < wv ? red[w] : 0;
        ndt += red[w];
    }
    int os = oslot;
#pragma unroll
    for (int u = 0; u < DR_SMAX / DR_NT; ++u) {
        if (!hq[u]) continue;
        E8[os].nd = nd;
        nd += !mydup[u];
        ++os;
    }
    if (tid == 0) {
        DrRow d;
        d.base = base;
        d.r = r;
        d.bs = bL.x;
        d.L = (int)L;
        d.nu = nu;
        d.aL = g.vA[a0 + jl];
        rows[h] = d;
        g.rnnz[r] = (int)L + ndt;
        soff[r] = -1;  // (the compaction skips the row: k_rows_dr_fill writes it into C)
        if (enq) {     // (more DR rows than k_rows_dr_group sorts: a chunk per row and range)
            ord[h] = h;
            const int nch = (int)((L + DR_CH - 1) / DR_CH);
            const int c0 = atomicAdd(nchunk, nch);
            for (int c = 0; c < nch; ++c) chunks[c0 + c] = make_int4(h, 1, c * DR_CH, 0);
        }
    }
}

// one workgroup: the DR rows sorted by their run (B position) -> ord; a run's
// rows (mawi: every hub neighbour holds the hub's whole B row) cut into blocks
// of DR_GR, each block's chunks one per DR_CH range of the run -- so the fill
// reads the run once per block, not once per row (149 mawi rows re-read a
// 120 MB run: 18.7 GB of fetch beside 19.4 GB of writes, r5p).  A run's chunks
// are range-major (the blocks of one range adjacent).
__global__ __launch_bounds__(DR_NT) void k_rows_dr_group(const DrRow *rows, const int *ndrp, int *ord, int4 *chunks,
                                                         int *nchunk) {
    constexpr int NW = DR_NT / 64, PT = DR_GMAX / DR_NT;
    __shared__ unsigned long long sk[DR_GMAX];  // (run start << 32 | row slot), sorted
    __shared__ int red[NW];
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int n = *ndrp;
    int npow = 1;
    while (npow < n) npow <<= 1;
    for (int q = tid; q < npow; q += DR_NT)
        sk[q] = q < n ? ((unsigned long long)(unsigned)rows[q].bs << 32) | (unsigned)q : ~0ull;
    __syncthreads();
    for (int K = 2; K <= npow; K <<= 1)
        for (int J = K >> 1; J > 0; J >>= 1) {
            for (int i = tid; i < npow; i += DR_NT) {
                const int ij = i ^ J;
                if (ij > i) {
                    const unsigned long long a = sk[i], b = sk[ij];
                    const bool asc = (i & K) == 0;
                    if ((a > b) == asc) {
                        sk[i] = b;
                        sk[ij] = a;
                    }
                }
            }
            __syncthreads();
        }
    // PT consecutive positions per thread: block heads, their chunk counts
    int cnt[PT], tot = 0;
#pragma unroll
    for (int u = 0; u < PT; ++u) {
        const int i = tid * PT + u;
        cnt[u] = 0;
        if (i >= n) continue;
        const unsigned run = (unsigned)(sk[i] >> 32);
        int lo = 0, hi = i;  // the run's first position
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((unsigned)(sk[mid] >> 32) < run) lo = mid + 1; else hi = mid;
        }
        if ((i - lo) % DR_GR == 0) cnt[u] = (rows[(unsigned)sk[i]].L + DR_CH - 1) / DR_CH;
        tot += cnt[u];
    }
    const int inc = wave_incl_scan_dpp(tot);
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    int o = inc - tot, all = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        o += w < wv ? red[w] : 0;
        all += red[w];
    }
#pragma unroll
    for (int u = 0; u < PT; ++u) {
        const int i = tid * PT + u;
        if (i < n) ord[i] = (int)(unsigned)sk[i];
        if (!cnt[u]) continue;
        const unsigned run = (unsigned)(sk[i] >> 32);
        int lo = 0, hi = i;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((unsigned)(sk[mid] >> 32) < run) lo = mid + 1; else hi = mid;
        }
        int e = i + 1, eh = n;  // past the run's last position
        while (e < eh) {
            const int mid = (e + eh) >> 1;
            if ((unsigned)(sk[mid] >> 32) <= run) e = mid + 1; else eh = mid;
        }
        const int R = cnt[u], S = (e - lo + DR_GR - 1) / DR_GR, sb = (i - lo) / DR_GR;
        const int gbase = o - sb * R;
        const int nr = min(DR_GR, e - i);
        for (int c = 0; c < R; ++c) chunks[gbase + c * S + sb] = make_int4(i, nr, c * DR_CH, 0);
        o += R;
    }
    if (tid == 0) *nchunk = all;
}

// a chunk: DR_CH elements of one run, held in registers, written for each of
// the chunk's rows (consecutive in ord, all of that run); a persistent grid
// (the chunk count is known on the device only)
constexpr int DR_FU = DR_CH / DR_NT;
__global__ __launch_bounds__(DR_NT) void k_rows_dr_fill(RowsArgs g, const int *Crp, int *Ccol, double *Cval,
                                                        const DrRow *rows, const DrEnt *ents, const int *ord,
                                                        const int4 *chunks, const int *nchunk) {
    __shared__ int sp[DR_SMAX];   // a row's S entries in the range: insertion points
    __shared__ int snd[DR_SMAX];  // inserted columns before each
    __shared__ unsigned char sdup[DR_SMAX];
    __shared__ double sval[DR_SMAX];
    __shared__ int r_lo[DR_GR], r_hi[DR_GR], r_nd0[DR_GR], r_h[DR_GR], r_out[DR_GR];
    __shared__ double r_a[DR_GR];
    const int tid = threadIdx.x;
    const int nck = *nchunk;
    for (int q = blockIdx.x; q < nck; q += gridDim.x) {  // (workgroup-uniform)
        const int4 ch = chunks[q];  // {first position in ord, rows, range start, -}
        const int nr = ch.y, i0 = ch.z;
        const DrRow d0 = rows[ord[ch.x]];
        const int i1 = min(d0.L, i0 + DR_CH);
        const bool last = i1 == d0.L;
        // the range, loads issued first (read once for the chunk's rows)
        int c[DR_FU];
        double v[DR_FU];
#pragma unroll
        for (int u = 0; u < DR_FU; ++u) {
            const int i = i0 + u * DR_NT + tid;
            c[u] = i < i1 ? g.Bcol[d0.bs + i] : 0;
            v[u] = i < i1 ? g.Bval[d0.bs + i] : 0.0;
        }
        // per row, two lanes: its S entries with insertion point in [i0, i1)
        // (the last range: [i0, L]), the inserted columns before the range
        if (tid < 2 * nr) {
            const int j = tid >> 1, hi_side = tid & 1;
            const int h = ord[ch.x + j];
            const DrRow d = rows[h];
            const DrEnt *const E8 = ents + (long)h * DR_SMAX;
            const int key = hi_side ? (last ? d.L + 1 : i1) : i0;
            int lo = 0, hi = d.nu;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (E8[mid].p < key) lo = mid + 1; else hi = mid;
            }
            if (hi_side) {
                r_hi[j] = lo;
            } else {
                r_lo[j] = lo;
                r_h[j] = h;
                r_out[j] = Crp[d.r];
                r_a[j] = d.aL;
                r_nd0[j] = lo < d.nu ? E8[lo].nd : (d.nu ? E8[d.nu - 1].nd + !E8[d.nu - 1].dup : 0);
            }
        }
        __syncthreads();
        for (int j = 0; j < nr; ++j) {
            const int elo = r_lo[j], ne = r_hi[j] - elo, nd0 = r_nd0[j];
            int *const Ocol = Ccol + r_out[j];
            double *const Oval = Cval + r_out[j];
            const double aL = r_a[j];
            // (plain stores: nontemporal ones 0.8 ms slower on mawi's 19 GB of C, r5r)
            if (ne == 0) {  // (most rows' ranges: the run shifted by the inserted columns before it)
#pragma unroll
                for (int u = 0; u < DR_FU; ++u) {
                    const int i = i0 + u * DR_NT + tid;
                    if (i < i1) {
                        Ocol[i + nd0] = c[u];
                        Oval[i + nd0] = aL * v[u];
                    }
                }
                continue;
            }
            const DrEnt *const E8 = ents + (long)r_h[j] * DR_SMAX;
            for (int t = tid; t < ne; t += DR_NT) {
                const DrEnt e = E8[elo + t];
                sp[t] = e.p;
                snd[t] = e.nd;
                sdup[t] = e.dup;
                sval[t] = e.val;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < DR_FU; ++u) {
                const int i = i0 + u * DR_NT + tid;
                if (i >= i1) break;
                double x = aL * v[u];
                // entries with p <= i: the count t; the inserted ones before i = nd of entry t
                int lo = 0, hi = ne;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (sp[mid] <= i) lo = mid + 1; else hi = mid;
                }
                const int ins = lo < ne ? snd[lo] : snd[ne - 1] + !sdup[ne - 1];
                if (lo > 0 && sp[lo - 1] == i && sdup[lo - 1]) x += sval[lo - 1];
                Ocol[i + ins] = c[u];
                Oval[i + ins] = x;
            }
            for (int t = tid; t < ne; t += DR_NT)
                if (!sdup[t]) {
                    const DrEnt e = E8[elo + t];
                    Ocol[e.p + e.nd] = e.col;
                    Oval[e.p + e.nd] = e.val;
                }
            __syncthreads();  // (the LDS tables: the next row's)
        }
        __syncthreads();  // (the row tables: the next chunk's)
    }
}

// chunks of CP_CH output positions (a workgroup each, consecutive lanes on
// consecutive positions): the chunk's rows from cfirst (the row holding each
// chunk's first position), each nonempty row marks its first position in LDS, a
// running max gives every position its row.

__global__ __launch_bounds__(WG) void k_rows_cfirst(int m, const int *Crp, long nch, int *cfirst) {
    // a thread per chunk: the last row starting at or before its first position
    // (a row per thread walked its chunks serially: 83 us on the mawi prefix,
    // 3,360 rows of ~445 K nonzeros)
    for (long b = (long)blockIdx.x * WG + threadIdx.x; b < nch; b += (long)gridDim.x * WG) {
        const long long pos = b * CP_CH;
        int lo = 0, hi = m;  // the answer lies in [lo, hi): Crp[lo] <= pos
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if ((long long)Crp[mid] <= pos) lo = mid; else hi = mid;
        }
        cfirst[b] = lo;
    }
}

// (the grid may cover more chunks than nnz(C) has -- sized by the products,
// so that no host round trip waits for nnz: the surplus workgroups exit)
__global__ __launch_bounds__(WG) void k_rows_compact(int m, const int *cfirst, const long long *soff, const int *Crp,
                                                     const int *Scol, const double *Sval, int *Ccol, double *Cval) {
    __shared__ int rowof[CP_CH];
    __shared__ int red[WAVES];
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int nnz = Crp[m];
    const int c0 = blockIdx.x * CP_CH;
    if (c0 >= nnz) return;  // (workgroup-uniform)
    const int n = min(CP_CH, nnz - c0);
    const int rf = cfirst[blockIdx.x];
    const int rl = c0 + CP_CH < nnz ? cfirst[blockIdx.x + 1] : m - 1;
    if (rf == rl && soff[rf] < 0) return;  // (inside one row written elsewhere: windowed / dominant-run)
    for (int i = tid; i < CP_CH; i += WG) rowof[i] = i == 0 ? rf : -1;
    __syncthreads();
    for (int r = rf + 1 + tid; r <= rl; r += WG) {
        const int s = Crp[r];
        if (s < c0 + n && Crp[r + 1] > s) rowof[s - c0] = r;
    }
    __syncthreads();
    // running max over the chunk: 8 positions per thread, then the threads
    constexpr int PT = CP_CH / WG;
    int loc[PT], mx = -1;
#pragma unroll
    for (int u = 0; u < PT; ++u) {
        mx = max(mx, rowof[tid * PT + u]);
        loc[u] = mx;
    }
    int inc = wave_incl_max(mx);
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    int carry = __shfl_up(inc, 1, 64);
    if (lane == 0) carry = -1;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) carry = w < wv ? max(carry, red[w]) : carry;
#pragma unroll
    for (int u = 0; u < PT; ++u) rowof[tid * PT + u] = max(carry, loc[u]);
    __syncthreads();
    // each thread's PT positions: their rows' offsets, then every load, then
    // every store (a windowed row's positions, soff < 0, are k_rows_wunit<1>'s)
    long long src[PT];
    bool ok[PT];
#pragma unroll
    for (int u = 0; u < PT; ++u) {
        const int i = u * WG + tid;
        ok[u] = i < n;
        const int r = ok[u] ? rowof[i] : 0;
        const long long so = ok[u] ? soff[r] : -1;
        ok[u] = so >= 0;
        src[u] = ok[u] ? so + (c0 + i - Crp[r]) : 0;
    }
    int cv[PT];
    double xv[PT];
#pragma unroll
    for (int u = 0; u < PT; ++u)
        if (ok[u]) {  // (streamed: staging read once, C not re-read by this call)
            cv[u] = __builtin_nontemporal_load(Scol + src[u]);
            xv[u] = __builtin_nontemporal_load(Sval + src[u]);
        }
#pragma unroll
    for (int u = 0; u < PT; ++u)
        if (ok[u]) {
            __builtin_nontemporal_store(cv[u], Ccol + c0 + u * WG + tid);
            __builtin_nontemporal_store(xv[u], Cval + c0 + u * WG + tid);
        }
}

// Two-launch exclusive scans (tile sums, then an apply that adds up the earlier
// tiles' sums) for the other CSR paths; TSG_ERR_UNSUPPORTED past RS_INLINE_MAX
// tiles (the caller then takes the generic scan).  Row pointers: n = m + 1,
// nnz(C) (the last value) into the host-mapped *hnnz_dev.
int dev_scan_i64_fused(Context &cx, long long *a, long n, hipStream_t s) {
    const long nt = (n + RS_TILE - 1) / RS_TILE;
    if (n <= 0) return TSG_OK;
    if (nt > RS_INLINE_MAX) return TSG_ERR_UNSUPPORTED;
    long long *part = nullptr;
    TSG_TRY(cx.get(&part, (size_t)nt));
    k_rows_count_sum<long long><<<(unsigned)nt, WG, 0, s>>>(a, n, part);
    k_rows_scan_apply<long long, false><<<(unsigned)nt, WG, 0, s>>>(a, n, part, nullptr, 0, nullptr);
    TSG_HIP(hipGetLastError());
    cx.put(part);  // (stream-ordered reuse)
    return TSG_OK;
}
int dev_scan_rows_fused(Context &cx, int *rp, int m, int *hnnz_dev, hipStream_t s) {
    const long n = (long)m + 1, nt = (n + RS_TILE - 1) / RS_TILE;
    if (nt > RS_INLINE_MAX) return TSG_ERR_UNSUPPORTED;
    int *part = nullptr;
    TSG_TRY(cx.get(&part, (size_t)nt));
    k_rows_count_sum<int><<<(unsigned)nt, WG, 0, s>>>(rp, n, part);
    k_rows_scan_apply<int, true><<<(unsigned)nt, WG, 0, s>>>(rp, n, part, nullptr, m, hnnz_dev);
    TSG_HIP(hipGetLastError());
    cx.put(part);  // (stream-ordered reuse)
    return TSG_OK;
}

// Setup (stream-ordered, no host round trip): the entry table, its scan and the
// classes; counts and statistics land in cx.pinned64[0..7) once the stream is synced.
int dev_rows_setup_async(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, RowsPlan &p, hipStream_t s,
                         SortedShares *sh) {
    static_assert(NCLS <= 8, "class counts in cls[0..8)");
    const int m = A.m;
    p = RowsPlan{};
    TSG_TRY(cx.get(&p.ebnd, (size_t)A.nnz + 1));
    TSG_TRY(cx.get(&p.E, (size_t)A.nnz + 1));
    TSG_TRY(cx.get(&p.lists, (size_t)NCLS * (m > 0 ? m : 1)));
    TSG_TRY(cx.get(&p.soff, (size_t)m + 1));
    // class counts [0..8), 5 u64 statistics [8..18), hub rows' cursors [18..22), the one-walk
    // rows' scratch products (u64) [24..26) and its cursor [26..28)
    TSG_TRY(cx.get(&p.cls, 32));
    TSG_TRY(cx.get(&p.rowpointer, (size_t)m + 1));
    unsigned long long *hst = reinterpret_cast<unsigned long long *>(p.cls + 8);
    const long ntile = ((long)A.nnz + 1 + RS_TILE - 1) / RS_TILE;
    if (ntile <= RS_INLINE_MAX) {  // entry table + tile sums, then the apply: two launches
        long long *part = nullptr;
        TSG_TRY(cx.get(&part, (size_t)ntile));
        k_rows_entries_sum<<<(unsigned)ntile, WG, 0, s>>>(A.columnindex, A.nnz, B.rowpointer, p.ebnd, p.E, p.cls,
                                                          part);
        k_rows_scan_apply<long long, false><<<(unsigned)ntile, WG, 0, s>>>(p.E, (long)A.nnz + 1, part, nullptr, 0,
                                                                           nullptr);
        TSG_HIP(hipGetLastError());
        cx.put(part);  // (stream-ordered reuse)
    } else {
        k_rows_entries<<<grid_for((long)A.nnz + 1, WG, 16384), WG, 0, s>>>(A.columnindex, A.nnz, B.rowpointer,
                                                                          p.ebnd, p.E, p.cls);
        TSG_HIP(hipGetLastError());
        TSG_TRY(scan_exclusive_i64(cx, p.E, (long)A.nnz + 1, s));
    }
    // (one workgroup at least: it writes the statistics and rowpointer[m])
    k_rows_bin<<<max(1, (m + BIN_ROWS - 1) / BIN_ROWS), WG, 0, s>>>(
        A.rowpointer, m, p.E, p.E + A.nnz, p.rowpointer, p.lists, p.cls, p.soff, hst, sh ? sh->part : nullptr,
        sh ? sh->nb : 0, sh ? sh->dflag : nullptr);
    TSG_HIP(hipGetLastError());
    if (sh) {
        cx.put(sh->part);  // (stream-ordered reuse)
        *sh = SortedShares{};
    }
    TSG_HIP(hipMemcpyAsync(cx.pinned64, p.cls, 26 * sizeof(int), hipMemcpyDeviceToHost, s));
    return TSG_OK;
}

void dev_rows_setup_read(Context &cx, RowsPlan &p) {
    for (int t = 0; t < NCLS; ++t) p.ncls[t] = reinterpret_cast<const int *>(cx.pinned64)[t];
    p.hprod = cx.pinned64[4];
    p.pmax = cx.pinned64[5];
    p.products = cx.pinned64[6];
    p.hubprod = cx.pinned64[7];
    p.hk = cx.pinned64[8];
    p.hbig = cx.pinned64[12];
}

// routing: every product whose B rows are strictly column-sorted (class H's
// rows take the one-walk bitmap, dominant-run or windowed kernels) -- unless a
// row holds more than 2^31 - 1 products (the class-H kernels count a row's
// products in int): such products go to the staged tile pipeline instead of
// failing (a forced TSG_PATH=rows still returns TSG_ERR_UNSUPPORTED for them)
bool dev_rows_accept(const RowsPlan &p) { return p.pmax <= 0x7fffffffLL; }

void dev_rows_release(Context &cx, RowsPlan &p) {
    void *ps[] = {p.ebnd, p.E, p.lists, p.soff, p.cls, p.rowpointer};
    for (void *q : ps) cx.put(q);
    p = RowsPlan{};
}

// CSR in -> CSR out from a setup (B's rows column-sorted; the caller checked);
// consumes the plan.  ev (optional): 1 set up | 4..5 the row kernels | 3 end
int dev_rows_run(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, RowsPlan &p, tsg_dev_csr &C,
                 tsg_stats *st, hipStream_t s, hipEvent_t *ev) {
    const int m = A.m;
    // (a row's products are counted in int inside the class-H kernels: a row past
    // 2^31 - 1 products is refused rather than wrapped)
    if (p.pmax > 0x7fffffffLL) {
        dev_rows_release(cx, p);
        return TSG_ERR_UNSUPPORTED;
    }
    C = tsg_dev_csr{};
    C.m = m;
    C.n = B.n;
    C.rowpointer = p.rowpointer;
    p.rowpointer = nullptr;  // (now C's)
    int2 *ebnd = p.ebnd;
    long long *E = p.E, *soff = p.soff;
    int4 *lists = p.lists;
    const long long products = p.products;
    int ncls[NCLS];
    for (int t = 0; t < NCLS; ++t) ncls[t] = p.ncls[t];
    // (exact row counts first, so that the classes write C in place, measured
    // slower on webbase twice: round 3's per-row count kernels took 318 us
    // against the 300 us compaction they save; round 5's several-rows-per-
    // workgroup LDS hash counts of the merge classes (k_rows_mcount, the staged
    // S/H rows copied by row) took 326 us, e2e 1.56 vs 1.29 ms --
    // tools/archive/rows_direct_hashcount.patch; the staging + compaction stays)
    int *Scol = nullptr;
    double *Sval = nullptr;
    TSG_TRY(cx.get(&Scol, (size_t)products + 1));
    TSG_TRY(cx.get(&Sval, (size_t)products + 1));
    if (ev && cx.stage_ev) TSG_HIP(hipEventRecord(ev[1], s));
    if (ev) TSG_HIP(hipEventRecord(ev[4], s));
#ifdef TSG_ROWS_PROF
    unsigned long long *dprof = nullptr;
    TSG_HIP(hipGetSymbolAddress((void **)&dprof, HIP_SYMBOL(g_rows_prof)));
    TSG_HIP(hipMemsetAsync(dprof, 0, sizeof(unsigned long long) * 3 * 256 * 12, s));
#endif
    RowsArgs g{A.rowpointer, A.value, ebnd, E, B.columnindex, B.value, nullptr, 0, C.rowpointer, Scol, Sval};
    // the classes in turn on the call's stream, heaviest first: class H alone
    // (its workgroups take a whole CU's LDS and starved behind the short rows'
    // workgroups when launched beside them), then M4 .. S16.  (The classes on
    // four streams, forked and joined, measured the same: the phase is bound by
    // the resident waves' latency chains, and the join cost ~26 us.)
    auto launch = [&](int c, auto kern, int grid, int nt, hipStream_t st) -> int {
        if (ncls[c] == 0) return TSG_OK;
        g.list = lists + (long)c * m;
        g.nrows = ncls[c];
        kern<<<grid, nt, 0, st>>>(g);
        TSG_HIP(hipGetLastError());
        return TSG_OK;
    };
    auto launch_m = [&](int c, auto kern, int grid, int nt, hipStream_t st) -> int {
        if (ncls[c] == 0) return TSG_OK;
        g.list = lists + (long)c * m;
        g.nrows = ncls[c];
        kern<<<grid, nt, 0, st>>>(g);
        TSG_HIP(hipGetLastError());
        return TSG_OK;
    };
    // the merge classes are persistent: one resident wave of workgroups
    if (ncls[7] >= 2 && ncls[7] <= OH_MAX) {
        k_rows_order_h<<<1, OH_NT, 0, s>>>(E, p.cls, lists + (long)(NCLS - 1) * m);
        TSG_HIP(hipGetLastError());
    }
    int *Oc = nullptr, *Or = nullptr;
    double *Ox = nullptr;
    DrRow *drows = nullptr;
    DrEnt *dents = nullptr;
    int4 *dchunks = nullptr;
    int *dord = nullptr;
    // windowed (W) rows' arrays: per class-H row, per unit, per chunk
    int *wnw = nullptr, *wnch = nullptr, *wlo = nullptr, *wwb = nullptr, *umap = nullptr;
    int *ucnt = nullptr, *ubo = nullptr, *ucount = nullptr, *uoff = nullptr, *ulist = nullptr, *ulist2 = nullptr,
        *lcnt = nullptr;  // (the lists' three sizes packed in one u64, 21 bits each)
    WUnit *urec = nullptr;
    long long *wmat = nullptr, *cmoff = nullptr;
    int *cbo = nullptr;
    unsigned long long *wst = nullptr;
    int4 *wchunks = nullptr;
    int nu = 0;
    long long drnch = 0;  // the dominant-run rows' fill chunks (launched after the row scan)
    RowsArgs g7 = g;  // (class H's list, for the windowed rows' gather after the row scan)
    if (ncls[7] > 0) {
        // class H: each kernel takes its rows of the class and its other
        // workgroups return at once
        const int n7 = ncls[7];
        g.list = lists + (long)7 * m;
        g.nrows = n7;
        long long wprod = 0, drprod = 0, ndr = 0, nmat = 0;
        int nc = 0;
        g7 = g;
        // rows past the one-walk kernel (hub rows, more than OW_RUNS runs, or a
        // span that may pass RH_SPAN): the plan sorts them into dominant-run and
        // windowed rows (one more host round trip: sizes of the unit and chunk lists)
        if (p.hubprod > 0 || p.hk > 0 || (long long)B.n > RH_SPAN) {
            TSG_TRY(cx.get(&wnw, (size_t)n7 + 1));
            TSG_TRY(cx.get(&wnch, (size_t)n7 + 1));
            TSG_TRY(cx.get(&wlo, (size_t)n7));
            TSG_TRY(cx.get(&wwb, (size_t)n7));
            TSG_TRY(cx.get(&wmat, (size_t)n7 + 1));
            TSG_TRY(cx.get(&wst, 4));
            TSG_HIP(hipMemsetAsync(wst, 0, 4 * sizeof(unsigned long long), s));
            // (W_UNIT products per unit: 4,096 measured equal, 16,384 / 32,768 slower)
            k_rows_wplan<<<n7, W_NT, 0, s>>>(g, B.n, W_UNIT, wnw, wnch, wlo, wwb, wmat,
                                             wst, soff);
            TSG_HIP(hipGetLastError());
            TSG_HIP(hipMemsetAsync(wnw + n7, 0, sizeof(int), s));
            TSG_HIP(hipMemsetAsync(wnch + n7, 0, sizeof(int), s));
            TSG_HIP(hipMemsetAsync(wmat + n7, 0, sizeof(long long), s));
            TSG_TRY(scan_exclusive_i32(cx, wnw, (long)n7 + 1, s));   // -> ubase
            TSG_TRY(scan_exclusive_i32(cx, wnch, (long)n7 + 1, s));  // -> cbase
            TSG_TRY(scan_exclusive_i64(cx, wmat, (long)n7 + 1, s));  // -> chunk x window offset matrix
            TSG_HIP(hipMemcpyAsync(cx.pinned64 + 16, wst, 3 * sizeof(long long), hipMemcpyDeviceToHost, s));
            TSG_HIP(hipMemcpyAsync(reinterpret_cast<int *>(cx.pinned64 + 20), wnw + n7, sizeof(int),
                                   hipMemcpyDeviceToHost, s));
            TSG_HIP(hipMemcpyAsync(reinterpret_cast<int *>(cx.pinned64 + 21), wnch + n7, sizeof(int),
                                   hipMemcpyDeviceToHost, s));
            TSG_HIP(hipMemcpyAsync(cx.pinned64 + 22, wmat + n7, sizeof(long long), hipMemcpyDeviceToHost, s));
            TSG_TRY(stream_wait(s));
            wprod = cx.pinned64[16];
            nmat = cx.pinned64[22];
            drprod = cx.pinned64[17];
            ndr = cx.pinned64[18];
            nu = *reinterpret_cast<const int *>(cx.pinned64 + 20);
            nc = *reinterpret_cast<const int *>(cx.pinned64 + 21);
        }
        if (nu > 0) {  // the windowed rows
            const int *ubase = wnw, *cbase = wnch;
            TSG_TRY(cx.get(&wchunks, (size_t)nc));
            TSG_TRY(cx.get(&cmoff, (size_t)nc));
            TSG_TRY(cx.get(&cbo, (size_t)nmat + 1));
            TSG_TRY(cx.get(&umap, (size_t)nu));
            TSG_TRY(cx.get(&ucnt, (size_t)nu));
            TSG_TRY(cx.get(&ubo, (size_t)nu));
            TSG_TRY(cx.get(&ucount, (size_t)nu));
            TSG_TRY(cx.get(&uoff, (size_t)nu));
            TSG_TRY(cx.get(&urec, (size_t)nu));
            TSG_TRY(cx.get(&ulist, (size_t)nu));
            TSG_TRY(cx.get(&ulist2, (size_t)nu));
            TSG_TRY(cx.get(&lcnt, 2));
            TSG_HIP(hipMemsetAsync(ucnt, 0, (size_t)nu * sizeof(int), s));
            TSG_HIP(hipMemsetAsync(lcnt, 0, 2 * sizeof(int), s));
            // (the run map of each walk step, not a binary search of the run table
            // per product: 2.75 vs 3.25 ms on the LiveJournal block)
            k_rows_wchunks<<<n7, WG, 0, s>>>(g, ubase, cbase, wmat, wchunks, cmoff, umap);
            TSG_HIP(hipGetLastError());
            k_rows_wcount<<<nc, W_NT, 0, s>>>(g, wchunks, cmoff, wlo, wwb, ubase, ucnt, cbo);
            TSG_HIP(hipGetLastError());
            k_rows_wscan<<<n7, W_NT, 0, s>>>(g, ubase, ucnt, ubo, nullptr, urec, wlo, wwb,
                                             nu < (1 << 21) ? ulist : nullptr, ulist2,
                                             reinterpret_cast<unsigned long long *>(lcnt), nu);
            TSG_HIP(hipGetLastError());
            k_rows_wscatter<<<nc, W_NT, 0, s>>>(g, wchunks, cmoff, wlo, wwb, ubase, ubo, cbo);
            TSG_HIP(hipGetLastError());
            k_rows_wunit<0, WU_NT0><<<nu, WU_NT0, 0, s>>>(g, urec, ucount, nullptr, nullptr, nullptr, nullptr);
            TSG_HIP(hipGetLastError());
            k_rows_wscan<<<n7, W_NT, 0, s>>>(g, ubase, ucount, uoff, g.rnnz);
            TSG_HIP(hipGetLastError());
#ifdef TSG_W_DUMP
            {  // (diagnostic) the units by window bits and products
                std::vector<WUnit> hr(nu);
                std::vector<int> hc(nu);
                TSG_HIP(hipMemcpyAsync(hr.data(), urec, sizeof(WUnit) * nu, hipMemcpyDeviceToHost, s));
                TSG_HIP(hipMemcpyAsync(hc.data(), ucount, sizeof(int) * nu, hipMemcpyDeviceToHost, s));
                TSG_TRY(stream_wait(s));
                long long cnt[19][8] = {}, pr[19][8] = {}, nz[19][8] = {};
                for (int u = 0; u < nu; ++u) {
                    int b = 0;
                    while (b < 7 && hr[u].n >= (64 << (2 * b))) ++b;
                    cnt[hr[u].wb][b]++;
                    pr[hr[u].wb][b] += hr[u].n;
                    nz[hr[u].wb][b] += hc[u];
                }
                fprintf(stderr, "W rows %d units %d chunks %d products %lld\n", n7, nu, nc, wprod);
                for (int w = 0; w < 19; ++w)
                    for (int b = 0; b < 8; ++b)
                        if (cnt[w][b])
                            fprintf(stderr, "  wb %2d n<%7d units %7lld products %10lld nnz %10lld\n", w,
                                    b < 7 ? (64 << (2 * b)) : -1, cnt[w][b], pr[w][b], nz[w][b]);
            }
#endif
        }
        if (p.hprod > wprod + drprod) {  // rows of the one-walk bitmap kernel
            if (p.hbig > 0) {  // one-walk rows past OW_CH products: their scratch
                TSG_TRY(cx.get(&Oc, (size_t)p.hbig));
                TSG_TRY(cx.get(&Ox, (size_t)p.hbig));
                TSG_TRY(cx.get(&Or, (size_t)p.hbig));
            }
            k_rows_bitmap<<<n7, RH_NT, 0, s>>>(g, Oc, Ox, Or, reinterpret_cast<unsigned long long *>(p.cls + 26));
            TSG_HIP(hipGetLastError());
        }
        if (drprod > 0) {  // hub rows with a dominant run
            const long long nch = drprod / DR_CH + ndr;
            TSG_TRY(cx.get(&drows, (size_t)ndr));
            TSG_TRY(cx.get(&dents, (size_t)ndr * DR_SMAX));
            TSG_TRY(cx.get(&dchunks, (size_t)nch));
            TSG_TRY(cx.get(&dord, (size_t)ndr));
            // (TSG_DR_PER_ROW: the per-row chunks also below DR_GMAX rows -- a test of that path)
            const bool grouped = ndr <= DR_GMAX && !getenv("TSG_DR_PER_ROW");
            k_rows_dr_prep<<<n7, DR_NT, 0, s>>>(g, soff, drows, dents, dord, dchunks, p.cls + 20, p.cls + 21,
                                                !grouped);
            TSG_HIP(hipGetLastError());
            if (grouped) {
                k_rows_dr_group<<<1, DR_NT, 0, s>>>(drows, p.cls + 21, dord, dchunks, p.cls + 20);
                TSG_HIP(hipGetLastError());
            }
            drnch = nch;
        }
    }
    auto classes = [&]() -> int {
        TSG_TRY(launch_m(6, k_rows_merge<M4_NT, M4_CAP, M4_RUNS>, ncls[6], M4_NT, s));
        TSG_TRY(launch_m(5, k_rows_merge<M3_NT, M3_CAP, M3_RUNS>, ncls[5], M3_NT, s));
        TSG_TRY(launch_m(4, k_rows_merge<M2_NT, M2_CAP, M2_RUNS>, ncls[4], M2_NT, s));
        TSG_TRY(launch_m(3, k_rows_merge<M1_NT, M1_CAP, M1_RUNS>, ncls[3], M1_NT, s));
        TSG_TRY(launch_m(2, k_rows_merge<M0_NT, M0_CAP, M0_RUNS>, ncls[2], M0_NT, s));
        TSG_TRY(launch(1, k_rows_small<64, S64_U>, (ncls[1] + WAVES * S64_U - 1) / (WAVES * S64_U), WG, s));
        TSG_TRY(launch(0, k_rows_small<16, S16_U>, (ncls[0] + 4 * WAVES * S16_U - 1) / (4 * WAVES * S16_U), WG, s));
        return TSG_OK;
    };
    // row counts -> row pointers -> C's arrays, with no host round trip: nnz(C)
    // <= products, so when the products fit int32 (and their 12 B each, beside
    // the staging's, stay within kRowsProductSizedC) the result arrays are sized
    // by them and nnz(C) comes back with the call's final synchronisation;
    // otherwise -- or when that allocation fails -- the checked scan reads nnz(C)
    // back first and C is sized exactly.
    long long nnz = 0;  // (C.rowpointer[m] = 0 from the binning kernel)
    // (TSG_ROWS_CHECKED_SCAN=1: the checked scan whatever the size -- tests take
    // the large products' path, with its fill lists, on small ones)
    const char *cs = getenv("TSG_ROWS_CHECKED_SCAN");
    bool small = products <= 0x7fffffffLL && products * 12 <= kRowsProductSizedC && !(cs && cs[0] == '1');
    long long cap = 0;
    // small with at most RS_INLINE_MAX tiles of row counts: one launch of tile
    // sums, then one apply that also fills the compaction's chunk table and
    // reports nnz(C) through the host-mapped pinned64[15] (no copy back)
    const long rtile = ((long)m + 1 + RS_TILE - 1) / RS_TILE;
    const bool fused_scan = small && rtile <= RS_INLINE_MAX;
    int *const hnnz = reinterpret_cast<int *>(cx.pinned64 + 15);
    int *const hl = reinterpret_cast<int *>(cx.pinned64 + 24);  // the fill lists' sizes (a packed u64)
    bool lknown = false;
    int *cfirst = nullptr;
    auto scan_alloc = [&]() -> int {
        if (small) {
            if (fused_scan) {
                int *part = nullptr;
                TSG_TRY(cx.get(&part, (size_t)rtile));
                // the apply fills the compaction's chunk table, a row's chunks by
                // one thread: fine for short rows, serial for hub rows (a 3.5 M-
                // nonzero LiveJournal row: 1.7 K chunks, ~50 us) -- past 2^20
                // products in a row, k_rows_cfirst (a thread per chunk) after it
                if (p.pmax <= (1LL << 20))
                    TSG_TRY(cx.get(&cfirst, (size_t)((products + CP_CH - 1) / CP_CH) + 1));
                k_rows_count_sum<int><<<(unsigned)rtile, WG, 0, s>>>(C.rowpointer, (long)m + 1, part);
                k_rows_scan_apply<int, true><<<(unsigned)rtile, WG, 0, s>>>(
                    C.rowpointer, (long)m + 1, part, cfirst, m, reinterpret_cast<int *>(cx.dpinned64 + 15));
                TSG_HIP(hipGetLastError());
                cx.put(part);  // (stream-ordered reuse)
            } else {
                TSG_TRY(scan_exclusive_i32(cx, C.rowpointer, (long)m + 1, s));
            }
            if (cx.get(&C.columnindex, (size_t)products + 1) != TSG_OK ||
                cx.get(&C.value, (size_t)products + 1) != TSG_OK) {
                cx.put(C.columnindex);
                C.columnindex = nullptr;
                small = false;  // (the scan's total is read back below)
                if (fused_scan) {
                    TSG_TRY(stream_wait(s));
                    C.nnz = *hnnz;
                } else {
                    TSG_TRY(read_i32(cx, C.rowpointer + m, &C.nnz, s));
                }
                nnz = C.nnz;
            }
        } else {  // the checked scan (nnz(C) past int32 fails)
            if (nu > 0 && nu < (1 << 21))  // (the fill lists' sizes come back with the scan's total)
                TSG_HIP(hipMemcpyAsync(hl, lcnt, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
            TSG_TRY(scan_exclusive_i32_total(cx, C.rowpointer, (long)m + 1, s, &nnz));
            lknown = nu > 0 && nu < (1 << 21);
            if (nnz > 0x7fffffffLL) return TSG_ERR_OVERFLOW;
        }
        cap = small ? products : nnz;
        if (!small) {
            TSG_TRY(cx.get(&C.columnindex, (size_t)cap + 1));
            TSG_TRY(cx.get(&C.value, (size_t)cap + 1));
        }
        return TSG_OK;
    };
    // the windowed rows' nonzeros straight into C (the compaction skips those rows)
    // and the dominant-run rows' (their counts exact since k_rows_dr_prep)
    auto wfill = [&]() -> int {
        if (nu > 0) {
            if (lknown) {
                // the list sizes came back with the checked scan's total: the bitmap
                // fill over its list (the longest units first), the sort fill over its
                const unsigned long long pk = *reinterpret_cast<const unsigned long long *>(hl);
                const int gs = (int)(pk & 0x1fffff), gh = (int)((pk >> 21) & 0x1fffff), gb = gh + (int)(pk >> 42);
                if (gb > 0)
                    k_rows_wunit<1, WU_NT><<<gb, WU_NT, 0, s>>>(g7, urec, ucount, uoff, C.rowpointer, C.columnindex,
                                                               C.value, ulist2, nu - 1, gh);
                if (gs > 0)
                    k_rows_wsort<<<gs, WS_NT, 0, s>>>(g7, urec, ulist, uoff, C.rowpointer, C.columnindex, C.value);
            } else {
                // (no read-back on this path: a host round trip of its own for the list
                // sizes, or grids of every unit with the surplus exiting, cost the
                // heaviest LiveJournal block 0.12-0.18 ms -- the bitmap fill takes all)
                k_rows_wunit<1, WU_NT><<<nu, WU_NT, 0, s>>>(g7, urec, ucount, uoff, C.rowpointer, C.columnindex,
                                                           C.value);
            }
            TSG_HIP(hipGetLastError());
        }
        if (drnch > 0) {
            // (persistent: the grouped chunk count, under drnch, is known on the device only)
            k_rows_dr_fill<<<(unsigned)std::min<long long>(drnch, 1024), DR_NT, 0, s>>>(
                g7, C.rowpointer, C.columnindex, C.value, drows, dents, dord, dchunks, p.cls + 20);
            TSG_HIP(hipGetLastError());
        }
        return TSG_OK;
    };
    {
        TSG_TRY(classes());
        // (the numeric phase: to the class kernels' end, or -- with windowed or
        // dominant-run rows, whose nonzeros go straight into C after the row
        // scan -- to the end of those fills, the scan included)
        const bool fills = nu > 0 || drnch > 0;
        if (ev && !fills) TSG_HIP(hipEventRecord(ev[5], s));
#ifdef TSG_ROWS_PROF
        {
            static unsigned long long raw[3 * 256 * 12];
            unsigned long long pr[36] = {};
            TSG_HIP(hipMemcpyAsync(raw, dprof, sizeof(raw), hipMemcpyDeviceToHost, s));
            TSG_TRY(stream_wait(s));
            for (int c = 0; c < 3; ++c)
                for (int b = 0; b < 256; ++b)
                    for (int k = 0; k < 12; ++k) pr[c * 12 + k] += raw[(c * 256 + b) * 12 + k];
            static const char *nm[3] = {"H", "M2-M4", "M0-M1"};
            for (int c = 0; c < 3; ++c) {
                const int cnt = c == 0 ? ncls[7] : c == 1 ? ncls[4] + ncls[5] + ncls[6] : ncls[2] + ncls[3];
                fprintf(stderr, "rows %s (%d rows) us/row:", nm[c], cnt);
                for (int k = 0; k < 12; ++k) fprintf(stderr, " %.2f", cnt ? pr[c * 12 + k] / 100.0 / cnt : 0.0);
                fprintf(stderr, "\n");
            }
        }
#endif
        TSG_TRY(scan_alloc());
        TSG_TRY(wfill());
        if (ev && fills) TSG_HIP(hipEventRecord(ev[5], s));
        if (cap > 0) {
            const int nch = (int)((cap + CP_CH - 1) / CP_CH);
            if (!cfirst) {  // (the fused scan filled it)
                TSG_TRY(cx.get(&cfirst, (size_t)nch + 1));
                k_rows_cfirst<<<grid_for(nch, WG, 16384), WG, 0, s>>>(m, C.rowpointer, (long)nch, cfirst);
                TSG_HIP(hipGetLastError());
            }
            k_rows_compact<<<nch, WG, 0, s>>>(m, cfirst, soff, C.rowpointer, Scol, Sval, C.columnindex, C.value);
        }
        TSG_HIP(hipGetLastError());
    }
    if (small && !fused_scan)
        TSG_HIP(hipMemcpyAsync(cx.pinned64 + 15, C.rowpointer + m, sizeof(int), hipMemcpyDeviceToHost, s));
    if (ev && cx.stage_ev) TSG_HIP(hipEventRecord(ev[3], s));
    TSG_TRY(stream_wait(s));
    if (small) nnz = *hnnz;
    C.nnz = (int)nnz;
    cx.put(cfirst);
    dev_rows_release(cx, p);
    cx.put(Scol);
    cx.put(Sval);
    {
        void *ws[] = {wnw, wnch, wlo, wwb, wmat, wst, wchunks, cmoff, cbo, umap, ucnt, ubo, ucount, uoff, urec,
                      ulist, ulist2, lcnt};
        for (void *q : ws) cx.put(q);
    }
    cx.put(Oc);
    cx.put(Ox);
    cx.put(Or);
    cx.put(drows);
    cx.put(dents);
    cx.put(dchunks);
    cx.put(dord);
    if (st) {
        st->nnzC = C.nnz;
        st->tile_products = products;
        st->numblkC = -1;
    }
    return TSG_OK;
}

}  // namespace tsg
