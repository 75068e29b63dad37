// tsg_band.hip -- banded path of the element TileSpGEMM for gfx950 (wave64):
// C = A*B, device CSR in -> device CSR out, B's rows column-sorted, every C
// row's reachable columns inside one window of <= BD_SPAN columns (banded /
// FEM-like operands such as cant).
//
// Reference semantics (paths under /root/reference/src): the same C as steps
// 1-3 + tile2csr (tilespgemm-cuda.h:279-2218, tile2csr.h:72-140); here the
// row's window plays the part of the reference's dense accumulator
// (tilespgemm-cuda.h:1954-2218, `dns`/`ful` bins): with the column span known,
// every element product lands at acc[col - lo] directly, so structure and
// values come from ONE walk over the products.
//
// One workgroup per C row:
//   * zero the row's window: an LDS fp64 accumulator acc[span] and one byte
//     per column;
//   * walk: a wave per A entry (its entries' B ranges loaded once, one per
//     lane; the next BD_U entries' B loads in flight during each group's LDS
//     updates; lane l takes B entries l, l+64, ...): ds_add_f64 of a*b into
//     acc[c - lo] and a plain byte store marking column c -- the row's C
//     structure and values together;
//   * the marks packed into a bitmap; a wave scan of its popcounts gives each
//     column its rank;
//   * the row's nonzeros are written in column order to a staging area at the
//     prefix of the window widths (a window bounds its row's nnz, and for
//     banded rows nearly equals it), and the row's nnz to the row pointers.
// A scan of the row counts gives the CSR row pointers and one streaming pass
// moves every row's run to its final place.  (A decoupled look-back over the
// rows in place of the staging measured 0.39 ms slower on cant: its chains of
// row-by-row resolution, not the walk, set the pace.)
#include "tsg_internal.h"
#include "tsg_dev_common.h"

#include <cstdlib>

namespace tsg {

namespace {

constexpr int BD_WG = 256;
constexpr int BD_SPAN = 2048;            // window columns per row: 16 KB fp64 + 256 B bitmap of LDS
constexpr int BD_WORDS = BD_SPAN / 32;   // bitmap words (= 64: one wave scans them)
constexpr int BD_SLOTS = 64;             // copies of the window statistics (k_band_stats)
constexpr int BD_U = 2;                  // entries per register set (two sets: 4 in flight)
static_assert(BD_WORDS == 64, "one bitmap word per lane");

}  // namespace

// Per C row: its column window [lo, hi] (first / last column of the B rows its
// entries reach; lo > hi for a row without products).  Statistics: bad[0] =
// rows whose window is wider than BD_SPAN, bad[1] = the widest window,
// bad[2..3] (u64) = the element products (they bound nnz(C)), bad[4..5] (u64)
// = the windows' columns in all.
__global__ __launch_bounds__(WG) void k_band_stats(const int *rpA, const int *ciA, int m, const int *rpB,
                                                   const int *ciB, int2 *win, long long *width, int *bad,
                                                   int2 *ebnd) {
    // 16 lanes per row, lane sl taking the row's entries sl, sl + 16, ... (four
    // entries' loads in flight): a row's ~64 entries (cant) are four dependent
    // load chains deep, not 64 (a thread per row walked them serially: 65 us)
    constexpr int G = 16, U = 4;
    __shared__ int red[2 * WAVES];
    __shared__ long long red64[WAVES];
    const int sl = threadIdx.x % G;
    int nbad = 0, wmax = 0;
    long long prod = 0, wsum = 0;
    const int rows_per_pass = gridDim.x * (WG / G);
    for (int r0 = blockIdx.x * (WG / G); r0 < m; r0 += rows_per_pass) {  // (workgroup-uniform)
        const int r = r0 + threadIdx.x / G;
        int lo = INT_MAX, hi = -1;
        long long q = 0;
        if (r < m) {
            const int a1 = rpA[r + 1];
            for (int a = rpA[r] + sl; a < a1; a += U * G) {
                int k[U];
#pragma unroll
                for (int u = 0; u < U; ++u) k[u] = a + u * G < a1 ? ciA[a + u * G] : -1;
                int b0[U], b1[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    b0[u] = k[u] >= 0 ? rpB[k[u]] : 0;
                    b1[u] = k[u] >= 0 ? rpB[k[u] + 1] : 0;
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (k[u] >= 0) ebnd[a + u * G] = make_int2(b0[u], b1[u]);  // (the banded path's entry table)
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (b1[u] > b0[u]) {
                        lo = min(lo, ciB[b0[u]]);
                        hi = max(hi, ciB[b1[u] - 1]);
                        q += b1[u] - b0[u];
                    }
                // this lane's share is already wider than a window: the row is
                // (its products and entry table only matter when every row fits,
                // and this one does not -- a hub row's 10^5 entries stop here)
                if (hi >= lo && hi - lo >= BD_SPAN) break;
            }
        }
#pragma unroll
        for (int d = G / 2; d > 0; d >>= 1) {
            lo = min(lo, __shfl_xor(lo, d, G));
            hi = max(hi, __shfl_xor(hi, d, G));
            q += __shfl_xor(q, d, G);
        }
        if (r < m && sl == 0) {
            const int w = hi >= lo ? hi - lo + 1 : 0;
            if (w > BD_SPAN) ++nbad;
            prod += q;
            wsum += w;
            wmax = max(wmax, w);
            win[r] = make_int2(lo, hi);
            width[r] = w;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) width[m] = 0;
    int mn = 0;
    block_minmax(mn, wmax, red);
    const int tb = block_sum(nbad, red);
    const long long tp = block_sum(prod, red64);
    const long long tw = block_sum(wsum, red64);
    if (threadIdx.x == 0) {  // (spread over BD_SLOTS copies: thousands of workgroups, no one hot address)
        int *const b = bad + 6 * (blockIdx.x % BD_SLOTS);
        if (tb) atomicAdd(&b[0], tb);
        if (wmax) atomicMax(&b[1], wmax);
        if (tp) atomicAdd(reinterpret_cast<unsigned long long *>(b + 2), (unsigned long long)tp);
        if (tw) atomicAdd(reinterpret_cast<unsigned long long *>(b + 4), (unsigned long long)tw);
    }
}

// the BD_SLOTS copies of the statistics into the first (the first wave); with
// spart, also B's sortedness shares (up to 4,096) summed by the workgroup into
// the host-mapped flag (the work of k_rows_sorted_final, in the same launch)
__global__ __launch_bounds__(WG) void k_band_stats_final(int *bad, const int *spart, int snb, int *sflag) {
    __shared__ long long red[WAVES];
    const int l = threadIdx.x;
    if (spart) {  // (workgroup-uniform)
        long long v = 0;
#pragma unroll 8
        for (int i = l; i < snb; i += WG) v += spart[i];
        v = block_sum(v, red);
        if (l == 0 && v != 0) __hip_atomic_store(sflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (l >= 64) return;
    int nb = l < BD_SLOTS ? bad[6 * l] : 0, wm = l < BD_SLOTS ? bad[6 * l + 1] : 0;
    long long tp = l < BD_SLOTS ? *reinterpret_cast<const long long *>(bad + 6 * l + 2) : 0;
    long long tw = l < BD_SLOTS ? *reinterpret_cast<const long long *>(bad + 6 * l + 4) : 0;
    nb = wave_sum(nb);
    wm = wave_last(wave_incl_max(wm));
    tp = wave_sum(tp);
    tw = wave_sum(tw);
    if (l == 0) {  // (one wave: its reads of every slot are done, the sums need them)
        bad[0] = nb;
        bad[1] = wm;
        *reinterpret_cast<long long *>(bad + 2) = tp;
        *reinterpret_cast<long long *>(bad + 4) = tw;
    }
}

struct BandArgs {
    const int *rpA;
    const double *vA;
    const int2 *ebnd;
    const int2 *win;
    const long long *soff;  // staging offset of each row (prefix of the window widths; null: r * BD_SPAN)
    const int *Bcol;
    const double *Bval;
    int *rnnz;              // nnz of each row (the row pointers after a scan)
    int *Scol;              // staging: each row's columns / values from soff[r]
    double *Sval;
    int m;                  // (rnnz[m] := 0, the scan's n+1 slot)
};

__global__ __launch_bounds__(BD_WG) void k_band_rows(BandArgs g) {
    __shared__ double acc[BD_SPAN];
    __shared__ __align__(16) unsigned char hit[BD_SPAN];      // column reached
    __shared__ __align__(16) unsigned char bmb[BD_SPAN / 8];  // the bitmap, 8 columns per byte
    __shared__ int wpre[BD_WORDS];
    const u32 *bm = reinterpret_cast<const u32 *>(bmb);
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const int r = xcd_item(blockIdx.x, gridDim.x);  // (neighbouring rows on one XCD: their B rows in its L2)
    const int2 w = g.win[r];
    const int lo = w.x, span = w.y >= w.x ? w.y - w.x + 1 : 0;
    const int nw = (span + 31) >> 5;
    for (int i = tid; i < span; i += BD_WG) acc[i] = 0.0;
    reinterpret_cast<uint2 *>(hit)[tid] = make_uint2(0u, 0u);  // 256 x 8 B = BD_SPAN bytes
    __syncthreads();
    // ---- the walk: each wave takes a contiguous share of the row's A entries,
    // so consecutive entries -- whose B rows in FEM operands are the dof
    // triplets of one node, with identical column sets (cant: rows 3u, 3u+1,
    // 3u+2) -- meet in one wave.  Lane l holds entries l and l + 64 of the
    // current B row (rows of <= 128 entries); while the next B row has the same
    // length and the same column on every lane (one ballot), its a*b is added in
    // registers, and only a change of pattern flushes the sums to the LDS
    // accumulator (ds_add_f64) and the hit bytes: one LDS atomic per column per
    // run of equal B rows instead of one per product.  B rows past 128 entries
    // go to the accumulator directly.  The next BD_U entries' B loads are in
    // flight during each group's work.
    const int a0 = g.rpA[r], a1 = g.rpA[r + 1];
    const int per = (a1 - a0 + 3) / 4;
    const int e0 = min(a1, a0 + wv * per), e1 = min(a1, a0 + (wv + 1) * per);
    int pc0 = -1, pc1 = -1, plen = -1;  // the pending pattern: columns of lanes l, l + 64; its length
    double px0 = 0.0, px1 = 0.0;
    auto put = [&](int c, double x) {
        atomicAdd(&acc[c], x);
        hit[c] = 1;  // (byte stores: an atomicOr into the bitmap put 32 lanes on one word)
    };
    auto flush = [&]() {
        if (pc0 >= 0) put(pc0, px0);
        if (pc1 >= 0) put(pc1, px1);
    };
    for (int base = e0; base < e1; base += 64) {  // wave-uniform
        const int my = base + lane;
        int2 me = make_int2(0, 0);
        double mav = 0.0;
        if (my < e1) {
            me = g.ebnd[my];
            mav = g.vA[my];
        }
        const int nj = min(64, e1 - base);
        // two register sets, a group of BD_U entries each: one loading while the
        // other is worked on (compile-time indices: the sets stay in VGPRs)
        int lnA[BD_U], cA0[BD_U], cA1[BD_U], lnB[BD_U], cB0[BD_U], cB1[BD_U];
        double xA0[BD_U], xA1[BD_U], xB0[BD_U], xB1[BD_U];
        auto load = [&](int j, int (&ln)[BD_U], int (&c0)[BD_U], int (&c1)[BD_U], double (&x0)[BD_U],
                        double (&x1)[BD_U]) {
#pragma unroll
            for (int k = 0; k < BD_U; ++k) {
                const int jj = min(j + k, 63);
                const int bs = __builtin_amdgcn_readlane(me.x, jj);
                const int be = j + k < nj ? __builtin_amdgcn_readlane(me.y, jj) : bs;
                const double av = __shfl(mav, jj, 64);
                ln[k] = be - bs;
                c0[k] = c1[k] = -1;
                x0[k] = x1[k] = 0.0;
                if (bs + lane < be) {
                    c0[k] = g.Bcol[bs + lane] - lo;
                    x0[k] = av * g.Bval[bs + lane];
                }
                if (bs + 64 + lane < be) {
                    c1[k] = g.Bcol[bs + 64 + lane] - lo;
                    x1[k] = av * g.Bval[bs + 64 + lane];
                }
            }
        };
        auto work = [&](int j, const int (&ln)[BD_U], const int (&c0)[BD_U], const int (&c1)[BD_U],
                        const double (&x0)[BD_U], const double (&x1)[BD_U]) {
#pragma unroll
            for (int k = 0; k < BD_U; ++k) {
                if (j + k >= nj) break;  // (wave-uniform)
                const int len = ln[k];
                if (len > 128) {  // a long B row: straight to the accumulator
                    flush();
                    pc0 = pc1 = plen = -1;
                    if (c0[k] >= 0) put(c0[k], x0[k]);
                    if (c1[k] >= 0) put(c1[k], x1[k]);
                    const int bs = __builtin_amdgcn_readlane(me.x, j + k);
                    const double av = __shfl(mav, j + k, 64);
                    for (int o = 128 + lane; o < len; o += 64) put(g.Bcol[bs + o] - lo, av * g.Bval[bs + o]);
                    continue;
                }
                const bool same = len == plen && __ballot(c0[k] != pc0 || c1[k] != pc1) == 0ull;
                if (same) {
                    px0 += x0[k];
                    px1 += x1[k];
                } else {
                    flush();
                    pc0 = c0[k];
                    pc1 = c1[k];
                    px0 = x0[k];
                    px1 = x1[k];
                    plen = len;
                }
            }
        };
        load(0, lnA, cA0, cA1, xA0, xA1);
        for (int j = 0; j < nj; j += 2 * BD_U) {  // (wave-uniform)
            if (j + BD_U < nj) load(j + BD_U, lnB, cB0, cB1, xB0, xB1);
            work(j, lnA, cA0, cA1, xA0, xA1);
            if (j + BD_U >= nj) break;
            if (j + 2 * BD_U < nj) load(j + 2 * BD_U, lnA, cA0, cA1, xA0, xA1);
            work(j + BD_U, lnB, cB0, cB1, xB0, xB1);
        }
    }
    flush();
    __syncthreads();
    {  // pack the marks: thread t's 8 columns [8t, 8t+8) -> bitmap byte t
        const uint2 v = reinterpret_cast<const uint2 *>(hit)[tid];
        const unsigned long long x = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
        bmb[tid] = (unsigned char)((x * 0x0102040810204080ull) >> 56);  // bit j = byte j (each 0 or 1)
    }
    __syncthreads();
    if (wv == 0) {  // ranks: popcount prefix of the bitmap words; the row's nnz
        const int cnt = lane < nw ? __popc(bm[lane]) : 0;
        const int inc = wave_incl_scan_dpp(cnt);
        wpre[lane] = inc - cnt;
        if (lane == 63) g.rnnz[r] = inc;
    }
    __syncthreads();
    // ---- the row's columns and values, in column order, to the staging area
    if (r == 0 && tid == 0) g.rnnz[g.m] = 0;
    // (the staging nontemporal, here and in k_band_compact: 208 MB on cant that
    // no later walk reads, kept out of the L2s that hold the B rows -- cant
    // 0.700 -> 0.651 ms, k_band_rows 500 -> 457 us; the same on the row-merge
    // classes' scattered row segments measured 0.6 ms slower)
    const long long E = g.soff ? g.soff[r] : (long long)r * BD_SPAN;
    for (int i = tid; i < span; i += BD_WG) {
        const u32 word = bm[i >> 5], bit = 1u << (i & 31);
        if (word & bit) {
            const long long pos = E + wpre[i >> 5] + __popc(word & (bit - 1u));
            __builtin_nontemporal_store(lo + i, g.Scol + pos);
            __builtin_nontemporal_store(acc[i], g.Sval + pos);
        }
    }
}

// every row's run from the staging area to its CSR place (wave per row)
__global__ __launch_bounds__(WG) void k_band_compact(int m, const long long *soff, const int *Crp, const int *Scol,
                                                     const double *Sval, int *Ccol, double *Cval) {
    for (int r = blockIdx.x * WAVES + wave_id(); r < m; r += gridDim.x * WAVES) {
        const long long s0 = soff ? soff[r] : (long long)r * BD_SPAN;
        const int d0 = Crp[r], n = Crp[r + 1] - d0;
        // (a cant row: ~280 nonzeros -- every load of a lane issued before its stores)
        int i = lane_id();
        for (; i + 192 < n; i += 256) {
            int c[4];
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                c[u] = __builtin_nontemporal_load(Scol + s0 + i + 64 * u);
                v[u] = __builtin_nontemporal_load(Sval + s0 + i + 64 * u);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                __builtin_nontemporal_store(c[u], Ccol + d0 + i + 64 * u);
                __builtin_nontemporal_store(v[u], Cval + d0 + i + 64 * u);
            }
        }
        for (; i < n; i += 64) {
            Ccol[d0 + i] = Scol[s0 + i];
            Cval[d0 + i] = Sval[s0 + i];
        }
    }
}

// routing: whether every C row's window fits BD_SPAN and the windows are dense
// (at least as many element products as window columns in all; `force` drops
// the density test).  Leaves the windows in *win_out (caller-owned, cx.put)
// when the answer is yes.
int dev_band_check(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, bool force, bool *ok, BandWin *bw,
                   hipStream_t s, SortedShares *sh) {
    *ok = false;
    *bw = BandWin{};
    if (A.m <= 0 || A.n != B.m) return sh ? dev_rows_sorted_finish(cx, *sh, s) : TSG_OK;
    int2 *win = nullptr, *ebnd = nullptr;
    long long *width = nullptr;
    int *bad = nullptr;
    TSG_TRY(cx.get(&win, (size_t)A.m));
    TSG_TRY(cx.get(&width, (size_t)A.m + 1));
    TSG_TRY(cx.get(&ebnd, (size_t)A.nnz + 1));
    TSG_TRY(cx.get(&bad, 6 * BD_SLOTS));
    TSG_HIP(hipMemsetAsync(bad, 0, 6 * BD_SLOTS * sizeof(int), s));
    k_band_stats<<<grid_for(A.m, WG / 16, 16384), WG, 0, s>>>(A.rowpointer, A.columnindex, A.m, B.rowpointer,
                                                        B.columnindex, win, width, bad, ebnd);
    const bool shares = sh && sh->part;
    k_band_stats_final<<<1, WG, 0, s>>>(bad, shares ? sh->part : nullptr, shares ? sh->nb : 0,
                                         shares ? sh->dflag : nullptr);
    TSG_HIP(hipGetLastError());
    if (sh) {
        cx.put(sh->part);  // (stream-ordered reuse)
        *sh = SortedShares{};
    }
    TSG_HIP(hipMemcpyAsync(cx.pinned + 8, bad, 6 * sizeof(int), hipMemcpyDeviceToHost, s));
    TSG_TRY(stream_wait(s));
    cx.put(bad);
    const long long products = *reinterpret_cast<const long long *>(cx.pinned + 10);
    const long long wcols = *reinterpret_cast<const long long *>(cx.pinned + 12);
    if (cx.pinned[8] == 0 && (force || products >= wcols)) {
        *ok = true;
        *bw = BandWin{win, width, products, wcols, ebnd};
    } else {
        cx.put(win);
        cx.put(width);
        cx.put(ebnd);
    }
    return TSG_OK;
}

__global__ __launch_bounds__(WG) void k_band_ebnd(const int *ciA, long nnzA, const int *rpB, int2 *ebnd) {
    for (long a = (long)blockIdx.x * WG + threadIdx.x; a < nnzA; a += (long)gridDim.x * WG) {
        const int k = ciA[a];
        ebnd[a] = make_int2(rpB[k], rpB[k + 1]);
    }
}

// CSR in -> CSR out for a banded product (windows from dev_band_check; their
// width array becomes the staging offsets).
// ev (optional): 0 start | 1 set up | 4..5 the row kernel | 3 end
int dev_spgemm_band(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, BandWin &bw, tsg_dev_csr &C,
                    tsg_stats *st, hipStream_t s, hipEvent_t *ev) {
    const int m = A.m;
    C = tsg_dev_csr{};
    C.m = m;
    C.n = B.n;
    if (ev) TSG_HIP(hipEventRecord(ev[0], s));
    int2 *ebnd = bw.ebnd;  // (filled by the window check's statistics kernel)
    bw.ebnd = nullptr;
    int *Scol = nullptr;
    double *Sval = nullptr;
    if (!ebnd) {
        TSG_TRY(cx.get(&ebnd, (size_t)A.nnz + 1));
        if (A.nnz > 0) k_band_ebnd<<<grid_for(A.nnz, WG, 16384), WG, 0, s>>>(A.columnindex, A.nnz, B.rowpointer, ebnd);
        TSG_HIP(hipGetLastError());
    }
    // staging: BD_SPAN slots per row while that stays within 2 GiB and within 4x
    // the window columns (no scan of the window widths: two launches fewer; cant:
    // 1.9x), else the widths' prefix (narrow windows: no near-2 GiB staging)
    const bool fixed = (long long)m * BD_SPAN * 12 <= (2LL << 30) && (long long)m * BD_SPAN <= 4 * bw.wcols;
    const long long slots = fixed ? (long long)m * BD_SPAN : bw.wcols;
    TSG_TRY(cx.get(&Scol, (size_t)slots + 1));
    TSG_TRY(cx.get(&Sval, (size_t)slots + 1));
    TSG_TRY(cx.get(&C.rowpointer, (size_t)m + 1));
    if (!fixed) {  // window widths -> staging offsets
        const int rc = dev_scan_i64_fused(cx, bw.width, (long)m + 1, s);
        if (rc == TSG_ERR_UNSUPPORTED) TSG_TRY(scan_exclusive_i64(cx, bw.width, (long)m + 1, s));
        else TSG_TRY(rc);
    }
    const long long *soff = fixed ? nullptr : bw.width;
    if (ev && cx.stage_ev) TSG_HIP(hipEventRecord(ev[1], s));
    if (ev) TSG_HIP(hipEventRecord(ev[4], s));
    if (m > 0) {
        BandArgs g{A.rowpointer, A.value, ebnd, bw.win, soff, B.columnindex, B.value, C.rowpointer, Scol, Sval, m};
        k_band_rows<<<m, BD_WG, 0, s>>>(g);
        TSG_HIP(hipGetLastError());
    }
    if (ev) TSG_HIP(hipEventRecord(ev[5], s));
    // row counts -> CSR row pointers (nnz(C) <= the window columns; past int32 fails).
    // While the window columns fit int32 and their 12 B each stay within
    // kRowsProductSizedC, C is sized by them: no read-back of nnz(C) before the
    // compaction (the fused scan stores it through host-mapped memory); else the
    // checked scan reads it back first and C is sized exactly.
    long long nnz = 0;
    if (m == 0) TSG_HIP(hipMemsetAsync(C.rowpointer + m, 0, sizeof(int), s));  // (else k_band_rows writes it)
    bool fused = bw.wcols <= 0x7fffffffLL && bw.wcols * 12 <= kRowsProductSizedC;
    int *const hnnz = reinterpret_cast<int *>(cx.pinned64 + 15);
    if (fused) {
        const int rc = dev_scan_rows_fused(cx, C.rowpointer, m, reinterpret_cast<int *>(cx.dpinned64 + 15), s);
        if (rc == TSG_ERR_UNSUPPORTED) fused = false;
        else TSG_TRY(rc);
    }
    if (fused && (cx.get(&C.columnindex, (size_t)bw.wcols + 1) != TSG_OK ||
                  cx.get(&C.value, (size_t)bw.wcols + 1) != TSG_OK)) {
        (void)hipGetLastError();
        cx.put(C.columnindex);
        C.columnindex = nullptr;
        TSG_TRY(stream_wait(s));  // (the fused scan's nnz(C), then C sized exactly)
        nnz = *hnnz;
        TSG_TRY(cx.get(&C.columnindex, (size_t)nnz + 1));
        TSG_TRY(cx.get(&C.value, (size_t)nnz + 1));
    } else if (!fused) {
        TSG_TRY(scan_exclusive_i32_total(cx, C.rowpointer, (long)m + 1, s, &nnz));
        if (nnz > 0x7fffffffLL) return TSG_ERR_OVERFLOW;
        TSG_TRY(cx.get(&C.columnindex, (size_t)nnz + 1));
        TSG_TRY(cx.get(&C.value, (size_t)nnz + 1));
    }
    if (m > 0)
        k_band_compact<<<grid_for(m, WAVES, 16384), WG, 0, s>>>(m, soff, C.rowpointer, Scol, Sval, C.columnindex,
                                                               C.value);
    TSG_HIP(hipGetLastError());
    if (ev && cx.stage_ev) TSG_HIP(hipEventRecord(ev[3], s));
    TSG_TRY(stream_wait(s));
    if (fused) nnz = *hnnz;
    if (nnz > 0x7fffffffLL) return TSG_ERR_OVERFLOW;
    C.nnz = (int)nnz;
    cx.put(ebnd);
    cx.put(Scol);
    cx.put(Sval);
    if (st) {
        st->nnzC = C.nnz;
        st->tile_products = bw.products;
        st->numblkC = -1;
    }
    return TSG_OK;
}

}  // namespace tsg
