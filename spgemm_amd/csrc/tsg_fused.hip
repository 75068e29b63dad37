// tsg_fused.hip -- the fused element-path TileSpGEMM for gfx950 (wave64):
// C = A*B, device CSR in -> device CSR out, B's rows column-sorted.
//
// Reference semantics (paths under /root/reference/src):
//   step 1  C tile structure            tilespgemm-cuda.h:279-392, nsparse :1171-1438
//   step 2  16-bit row masks of C tiles tilespgemm-cuda.h:394-773
//           + tile nnz scan             :2598-2604
//   step 3  values by mask-popcount rank tilespgemm-cuda.h:1273-2218
//   tile2csr                            tile2csr.h:72-140
//
// One persistent kernel does steps 1-3 and tile2csr for one UNIT of C at a
// time, with the unit's whole tile structure in LDS:
//   * a unit is a range of <= 256 C rows holding <= CAP element products, or
//     one column window of a heavy row; its CSR output is contiguous.
//   * walk 1 (symbolic): every element product (A entry, B entry) of the unit
//     inserts its C tile row-segment -- (row, tile column t = col/16), i.e. one
//     16-bit row of a 16x16 C tile -- into an LDS hash set and ORs its column
//     bit into that segment's mask; the product's slot and column bit are
//     cached in LDS (u16) for walk 2.
//   * the segments of each row are ordered by tile column (rank counting or an
//     LDS bitonic network); popcounts of the masks, scanned in that order, give
//     every segment its offset in the unit's CSR output.
//   * the unit's nnz is published with a decoupled look-back over the units
//     (ticketed in row order), which yields its global CSR offset and row
//     pointers -- no separate count pass, no device-wide scan of nnz(C).
//   * walk 2 (numeric): value products accumulate with ds_add_f64 at
//     offset + popcount(mask below the column) -- the reference step 3's rank
//     rule -- and the unit's columns and values are written once, coalesced.
//
// Heavy rows (more than CAP products) are cut into column windows: a
// per-row histogram of product columns over bins of <= 32768 columns (so a
// window holds <= 2048 tile columns) is merged into windows of <= CAP products
// (a single denser bin is a window of its own: its products then skip the slot
// cache and, past CAP nonzeros, accumulate in the output with global fp64
// atomics).
#include "tsg_internal.h"
#include "tsg_dev_common.h"

#include <cstdio>

namespace tsg {

namespace {

constexpr int FZ_CAP = 2048;          // element products per row unit
constexpr int FZ_H = 2 * FZ_CAP;      // hash slots (load <= 1/2)
constexpr int FZ_HBITS = 12;          // log2(FZ_H): slot bits of the product cache
constexpr int FZ_PS = FZ_CAP;         // product-slot cache entries
constexpr int FZ_NV = FZ_CAP;         // LDS value accumulator entries
constexpr int FZ_ROWS = 256;          // rows per row unit (row bits of a segment key)
constexpr int FZ_WG = 512;            // unit kernel workgroup (8 waves: 2 workgroups per CU)
constexpr int FZ_NW = FZ_WG / 64;
constexpr int FZ_SPT = FZ_H / 2 / FZ_WG;  // sorted positions per thread (S <= FZ_H / 2)
constexpr int FZ_SHORT = 8;           // product runs walked by their own thread
constexpr int FZ_SMALLROW = 64;       // rows ordered by rank counting (larger: bitonic)
constexpr int FZ_MAXBINS = 8192;      // heavy-row histogram bins
constexpr u32 FZ_EMPTY = 0xffffffffu;
constexpr unsigned long long FZ_AGG = 1ull << 62, FZ_INC = 2ull << 62, FZ_VAL = (1ull << 62) - 1;

static_assert(FZ_H == (1 << FZ_HBITS), "slot bits");
static_assert(FZ_HBITS + 4 <= 16, "product cache entry = slot | column bit << HBITS");

__device__ __forceinline__ u32 fz_hash(u32 key) { return (key * 0x9E3779B1u) >> (32 - FZ_HBITS); }

// exclusive scan / sum over the FZ_WG-thread workgroup; red needs FZ_NW entries
template <class T> __device__ __forceinline__ T fz_excl_scan(T x, T *total, T *red) {
    const T inc = wave_incl_scan(x);
    if (lane_id() == 63) red[wave_id()] = inc;
    __syncthreads();
    T off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < FZ_NW; ++w) {
        const T v = red[w];
        off += (w < wave_id()) ? v : T(0);
        tot += v;
    }
    __syncthreads();
    *total = tot;
    return off + inc - x;
}
template <class T> __device__ __forceinline__ T fz_sum(T x, T *red) {
    x = wave_sum(x);
    if (lane_id() == 0) red[wave_id()] = x;
    __syncthreads();
    T tot = 0;
#pragma unroll
    for (int w = 0; w < FZ_NW; ++w) tot += red[w];
    __syncthreads();
    return tot;
}

struct FzLds {
    u32 keys[FZ_H];     // segment key (row << 24 | tile column), FZ_EMPTY when free
    u32 info[FZ_H];     // walk 1: row-list index << 16 | mask;  walk 2: CSR offset << 16 | mask
    u16 pslot[FZ_PS];   // per product: slot | column bit << FZ_HBITS
    union {
        double vals[FZ_NV];   // walk 2 accumulator
        u32 sortv[FZ_H];      // per row, its segments (tile column << 8 | row), sorted in place
    } v;
    int rp[FZ_ROWS + 1];      // A row pointers of the unit's rows (absolute)
    int rseg[FZ_ROWS + 1];    // segments per row -> exclusive offsets into sortv
    int rnnz[FZ_ROWS + 1];    // nonzeros per row -> exclusive offsets in the unit's output
    int ebs[FZ_WG], ebe[FZ_WG];  // long product runs of the current entry batch
    int ep0[FZ_WG], elr[FZ_WG];
    double eav[FZ_WG];
    int nlong[FZ_NW];
    int big[FZ_ROWS];         // rows ordered by bitonic networks
    int nbig;
    int red[2 * FZ_NW];
    long long bc[2];
};

// ---- the unit's element products ------------------------------------------
// Entries a in [a0, a1) in batches of WG (one per thread): B range [bs, be)
// (narrowed to the column window), product index base = exclusive scan of the
// run lengths.  Runs <= FZ_SHORT are walked by their thread, longer ones by
// whole waves (lane l takes b = bs + l, bs + l + 64, ...: coalesced B reads).
// f(p, b, row, a_value) for every product p of the unit (same p in both walks).
template <bool VAL, class F>
__device__ __forceinline__ void fz_walk(FzLds &L, int a0, int a1, int nrows, const int2 *ebnd, const int *Bcol,
                                        const double *Aval, bool window, int clo, int chi, F &&f) {
    const int lane = lane_id(), wv = wave_id();
    int pbase = 0;
    for (int ab = a0; ab < a1; ab += FZ_WG) {
        const int a = ab + threadIdx.x;
        int bs = 0, be = 0, lr = 0;
        double av = 0.0;
        if (a < a1) {
            const int2 e = ebnd[a];
            bs = e.x;
            be = e.y;
            if (window) {
                bs = lower_bound_dev(Bcol, bs, be, clo);
                be = lower_bound_dev(Bcol, bs, be, chi);
            }
            lr = nrows > 1 ? owner_search(L.rp, nrows, a) : 0;
            if (VAL) av = Aval[a];
        }
        const int len = be - bs;
        int tot;
        const int off = fz_excl_scan(len, &tot, L.red) + pbase;
        const bool lng = len > FZ_SHORT;
        if (!lng)
            for (int j = 0; j < len; ++j) f(off + j, bs + j, lr, av);
        const u64 msk = __ballot(lng);
        if (lane == 0) L.nlong[wv] = __popcll(msk);
        __syncthreads();
        int base = 0, nl = 0;
#pragma unroll
        for (int w = 0; w < FZ_NW; ++w) {
            const int c = L.nlong[w];
            base += (w < wv) ? c : 0;
            nl += c;
        }
        if (lng) {
            const int pos = base + __builtin_amdgcn_mbcnt_hi((u32)(msk >> 32), __builtin_amdgcn_mbcnt_lo((u32)msk, 0u));
            L.ebs[pos] = bs;
            L.ebe[pos] = be;
            L.ep0[pos] = off;
            L.elr[pos] = lr;
            if (VAL) L.eav[pos] = av;
        }
        __syncthreads();
        for (int k = wv; k < nl; k += FZ_NW) {  // wave-uniform run
            const int sb = L.ebs[k], se = L.ebe[k], p0 = L.ep0[k], r = L.elr[k];
            const double ka = VAL ? L.eav[k] : 0.0;
            for (int b = sb + lane; b < se; b += 64) f(p0 + (b - sb), b, r, ka);
        }
        __syncthreads();  // the run list is rewritten by the next batch
        pbase += tot;
    }
}

__device__ __forceinline__ int fz_probe(const u32 *keys, u32 key) {
    u32 h = fz_hash(key);
    while (keys[h] != key) h = (h + 1) & (FZ_H - 1);
    return (int)h;
}

// ascending sort of n u32 keys in place by the calling wave (tid = lane, nt =
// 64, sync = wave_lds_sync) or workgroup (tid = threadIdx.x, nt = WG,
// __syncthreads): bitonic network, "flip" form (every comparator ascending, so
// positions >= n act as +inf and are never touched)
template <bool BLOCK>
__device__ __forceinline__ void fz_bitonic(u32 *a, int n) {
    const int tid = BLOCK ? (int)threadIdx.x : lane_id(), nt = BLOCK ? FZ_WG : 64;
    int lp = 0;
    while ((1 << lp) < n) ++lp;
    const int half = (1 << lp) >> 1;
    for (int lk = 1; lk <= lp; ++lk) {
        for (int lj = lk - 1; lj >= 0; --lj) {
            const int j = 1 << lj;
            for (int i = tid; i < half; i += nt) {
                const int blk = i >> lj, o = i & (j - 1);
                int lo, hi;
                if (lj == lk - 1) {  // flip: mirror pairs of each 2^lk block
                    lo = (blk << lk) + o;
                    hi = (blk << lk) + (1 << lk) - 1 - o;
                } else {
                    lo = (blk << (lj + 1)) + o;
                    hi = lo + j;
                }
                if (hi < n) {
                    const u32 x = a[lo], y = a[hi];
                    if (x > y) {
                        a[lo] = y;
                        a[hi] = x;
                    }
                }
            }
            if (BLOCK) __syncthreads(); else wave_lds_sync();
        }
    }
}

// Decoupled look-back over the units' nnz, in two halves so its latency hides
// behind the unit's ordering work (wave 0 only):
//   fz_publish: store the unit's aggregate (unit 0: its inclusive prefix) and
//     issue the loads of the 64 nearest predecessors' status words;
//   fz_resolve: consume them (re-reading any not yet published, and further
//     windows back until an inclusive prefix), publish the inclusive prefix and
//     return the unit's exclusive one.
__device__ __forceinline__ unsigned long long fz_ld(unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fz_st(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long fz_publish(unsigned long long *status, int u, long long n) {
    const int lane = lane_id();
    if (lane == 0) fz_st(&status[u], (u == 0 ? FZ_INC : FZ_AGG) | (unsigned long long)n);
    const int j = u - 1 - lane;
    return j >= 0 ? fz_ld(&status[j]) : FZ_INC;  // before unit 0: an inclusive 0
}

__device__ long long fz_resolve(unsigned long long *status, int u, long long n, unsigned long long st, int *fail) {
    if (u == 0) return 0;
    const int lane = lane_id();
    long long excl = 0;
    int j0 = u - 1;
    bool first = true;
    while (true) {
        const int j = j0 - lane;
        if (!first) st = j >= 0 ? fz_ld(&status[j]) : FZ_INC;
        first = false;
        // a predecessor that has not published yet: wait (ticket order guarantees
        // it is running); one that never publishes within 2 s of wall clock --
        // not a slow one, a fault -- fails the call instead of hanging it
        const unsigned long long w0 = wall_clock64();
        while ((st >> 62) == 0) {
            __builtin_amdgcn_s_sleep(1);
            st = fz_ld(&status[j]);
            if ((st >> 62) == 0 && wall_clock64() - w0 > 200000000ull) {  // (100 MHz wall clock: 2 s)
                atomicExch(fail, 2);
                st = FZ_INC;
            }
        }
        const u64 inc = __ballot((st >> 62) == 2);
        const long long val = (long long)(st & FZ_VAL);
        if (inc) {
            const int nearest = __ffsll((long long)inc) - 1;  // nearest predecessor with an inclusive prefix
            excl += wave_sum(lane <= nearest ? val : 0ll);
            break;
        }
        excl += wave_sum(val);
        j0 -= 64;
    }
    if (lane == 0) fz_st(&status[u], FZ_INC | (unsigned long long)(excl + n));
    return excl;
}

}  // namespace

// ---------------------------------------------------------------------------
// preparation: per A entry its B row range and run length; per row its
// products and class; unit counts; heavy-row windows; the unit table
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_fz_entries(const int *ciA, long nnzA, const int *rpB, int2 *ebnd,
                                                   long long *elen) {
    for (long a = (long)blockIdx.x * WG + threadIdx.x; a <= nnzA; a += (long)gridDim.x * WG) {
        if (a == nnzA) {
            elen[a] = 0;
            continue;
        }
        const int k = ciA[a];
        const int2 e = make_int2(rpB[k], rpB[k + 1]);
        ebnd[a] = e;
        elen[a] = e.y - e.x;
    }
}

// ucnt[r] = units starting at row r (heavy rows: filled by k_fz_heavy);
// heavy rows listed in hlist; ctr = {heavy rows, heavy products (u64 at +2)}.
// One wave per block of 256 rows packs them greedily: a row opens a new unit
// when the open unit's products would pass FZ_CAP, at the block start, and
// after a heavy row (units never span blocks: <= 256 rows each).
__global__ __launch_bounds__(WG) void k_fz_rows(const int *rpA, int m, const long long *cum, long nnzA, int *ucnt,
                                                int *hlist, int *ctr) {
    __shared__ int sp[WAVES][FZ_ROWS];  // per wave: its block's row products (-1: heavy)
    const int lane = lane_id(), wv = wave_id();
    const int nblk = (m + FZ_ROWS - 1) / FZ_ROWS;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ucnt[m] = 0;
        *reinterpret_cast<long long *>(ctr + 8) = cum[nnzA];  // the product total, read back with ctr
    }
    for (int blk0 = blockIdx.x * WAVES; blk0 < nblk; blk0 += gridDim.x * WAVES) {  // uniform per workgroup
        const int blk = blk0 + wv;
        if (blk < nblk) {
#pragma unroll
            for (int k = 0; k < FZ_ROWS / 64; ++k) {
                const int i = k * 64 + lane, r = blk * FZ_ROWS + i;
                int pv = 0;
                if (r < m) {
                    const long long q = cum[rpA[r + 1]] - cum[rpA[r]];
                    if (q > FZ_CAP) {  // heavy: column windows
                        const int pos = atomicAdd(&ctr[0], 1);
                        hlist[pos] = r;
                        atomicAdd(reinterpret_cast<unsigned long long *>(ctr + 2), (unsigned long long)q);
                        pv = -1;
                    } else {
                        pv = (int)q;
                    }
                }
                sp[wv][i] = pv;
            }
        }
        wave_lds_sync();
        if (blk < nblk && lane == 0) {
            // sequential greedy over the block's rows: rewrite sp[i] as the start flag
            int acc = FZ_CAP + 1;  // forces a start at the block's first light row
            const int nr = min(FZ_ROWS, m - blk * FZ_ROWS);
            for (int i = 0; i < nr; ++i) {
                const int pi = sp[wv][i];
                int st = 0;
                if (pi < 0) {
                    acc = FZ_CAP + 1;
                    st = -1;
                } else if (acc + pi > FZ_CAP) {
                    st = 1;
                    acc = pi;
                } else {
                    acc += pi;
                }
                sp[wv][i] = st;
            }
        }
        wave_lds_sync();
        if (blk < nblk) {
#pragma unroll
            for (int k = 0; k < FZ_ROWS / 64; ++k) {
                const int i = k * 64 + lane, r = blk * FZ_ROWS + i;
                if (r < m && sp[wv][i] >= 0) ucnt[r] = sp[wv][i];
            }
        }
        wave_lds_sync();
    }
}

// One workgroup per heavy row: histogram of its product columns over bins of
// binw columns (binw a multiple of 16, <= 32768), merged into windows of <=
// FZ_CAP products (a bin over FZ_CAP/2 is its own window).  Writes the
// window count to ucnt[r] and the windows (c_lo, c_hi, products) at wofs[r].
__global__ __launch_bounds__(WG) void k_fz_heavy(const int *hlist, const int *ctr, const int *rpA, const int2 *ebnd,
                                                 const int *Bcol, int n, int binw, int nbins, int *ucnt, int *wofs,
                                                 int4 *wtab, int *wtop) {
    __shared__ int hist[FZ_MAXBINS];
    __shared__ int ebs[WG], eoff[WG + 1];
    __shared__ int red[2 * WAVES];
    __shared__ int s_base;
    constexpr int half = FZ_CAP / 2;
    const int nh = ctr[0];
    for (int hi = blockIdx.x; hi < nh; hi += gridDim.x) {
        const int r = hlist[hi];
        for (int k = threadIdx.x; k < nbins; k += WG) hist[k] = 0;
        __syncthreads();
        const int a0 = rpA[r], a1 = rpA[r + 1];
        for (int ab = a0; ab < a1; ab += WG) {
            const int a = ab + threadIdx.x;
            int bs = 0, len = 0;
            if (a < a1) {
                const int2 e = ebnd[a];
                bs = e.x;
                len = e.y - e.x;
            }
            int tot;
            const int off = block_excl_scan(len, &tot, red);
            ebs[threadIdx.x] = bs;
            eoff[threadIdx.x] = off;
            __syncthreads();
            const int na = min(WG, a1 - ab);
            for (int q = threadIdx.x; q < tot; q += WG) {
                const int o = owner_search(eoff, na, q);
                atomicAdd(&hist[Bcol[ebs[o] + (q - eoff[o])] / binw], 1);
            }
            __syncthreads();
        }
        // windows: a start at bin k when k == 0, k or k-1 is dense (> half), or the
        // products before k cross a multiple of half
        constexpr int BPT = FZ_MAXBINS / WG;
        int cnt[BPT];
        int loc = 0;
#pragma unroll
        for (int j = 0; j < BPT; ++j) {
            const int k = threadIdx.x * BPT + j;
            cnt[j] = k < nbins ? hist[k] : 0;
            loc += cnt[j];
        }
        int tot;
        int pre = block_excl_scan(loc, &tot, red);
        // per bin: exclusive product prefix; start flags
        int starts = 0;
        int prev_cnt = threadIdx.x * BPT > 0 ? hist[threadIdx.x * BPT - 1] : 0;
        int prev_pre = pre - prev_cnt;
        bool st[BPT];
        {
            int p = pre;
#pragma unroll
            for (int j = 0; j < BPT; ++j) {
                const int k = threadIdx.x * BPT + j;
                bool s = false;
                if (k < nbins) {
                    s = k == 0 || cnt[j] > half || prev_cnt > half || (p / half) != (prev_pre / half);
                }
                st[j] = s;
                starts += s ? 1 : 0;
                prev_pre = p;
                prev_cnt = cnt[j];
                p += cnt[j];
            }
        }
        int nw;
        const int wpre = block_excl_scan(starts, &nw, red);
        if (threadIdx.x == 0) {
            s_base = atomicAdd(wtop, nw);
            ucnt[r] = nw;
            wofs[r] = s_base;
        }
        __syncthreads();
        // window w = (start bin, products); its end = the next window's start
        {
            int w = s_base + wpre, p = pre;
#pragma unroll
            for (int j = 0; j < BPT; ++j) {
                const int k = threadIdx.x * BPT + j;
                if (k < nbins && st[j]) {
                    wtab[w] = make_int4(r, k * binw, 0, p);  // .z (end) and .w (products) fixed below
                    ++w;
                }
                p += cnt[j];
            }
        }
        __syncthreads();
        for (int w0 = 0; w0 < nw; w0 += WG) {  // read a chunk, then rewrite it (.w: prefix -> count)
            const int w = w0 + threadIdx.x;
            int4 d = make_int4(0, 0, 0, 0), nx = d;
            if (w < nw) {
                d = wtab[s_base + w];
                nx = (w + 1 < nw) ? wtab[s_base + w + 1] : make_int4(r, n, 0, tot);
            }
            __syncthreads();
            if (w < nw) wtab[s_base + w] = make_int4(r, d.y, nx.y, nx.w - d.w);
            __syncthreads();
        }
    }
}

// unit table: utab[u] = (first row, c_lo, c_hi, products); c_lo = -1 for row units
__global__ __launch_bounds__(WG) void k_fz_fill(const int *ubase, int m, const int *wofs, const int4 *wtab,
                                                int4 *utab) {
    for (int r = blockIdx.x * WG + threadIdx.x; r < m; r += gridDim.x * WG) {
        const int u = ubase[r], c = ubase[r + 1] - u;
        if (c == 0) continue;
        if (c == 1 && (!wofs || wofs[r] < 0)) {
            utab[u] = make_int4(r, -1, 0, 0);
        } else {
            const int o = wofs[r];
            for (int k = 0; k < c; ++k) utab[u + k] = wtab[o + k];
        }
    }
}

// ---------------------------------------------------------------------------
// the fused unit kernel
// ---------------------------------------------------------------------------
struct FzArgs {
    const int *rpA, *ciA;
    const double *vA;
    const int2 *ebnd;
    const long long *cum;
    const int *Bcol;
    const double *Bval;
    const int4 *utab;
    const int *nunits_d;   // = ubase[m]
    int m;
    long long cap;         // allocated C entries
    unsigned long long *status;
    int *ticket;
    int *Crp, *Ccol;
    double *Cval;
    int *overflow;
    unsigned long long *nseg;  // C row-segments (non-empty 16-bit rows of C tiles)
    unsigned long long *prof;  // TSG_FZ_PROF builds: per-phase clock totals (9)
};

__global__ __launch_bounds__(FZ_WG) void k_fz_units(FzArgs g) {
    __shared__ FzLds L;
    __shared__ int s_u;
    const int tid = threadIdx.x;
#ifdef TSG_FZ_PROF
    unsigned long long prof_acc[9] = {}, prof_t = wall_clock64();
#define FZ_PROF(k)                                           \
    do {                                                     \
        const unsigned long long _t = wall_clock64();        \
        prof_acc[k] += _t - prof_t;                          \
        prof_t = _t;                                         \
    } while (0)
#else
#define FZ_PROF(k) \
    do {           \
    } while (0)
#endif
    const int nunits = *g.nunits_d;
    long long my_seg = 0;
    while (true) {
        if (tid == 0) s_u = atomicAdd(g.ticket, 1);
        __syncthreads();
        const int u = s_u;
        if (u >= nunits) break;
        FZ_PROF(0);
        const int4 d = g.utab[u];
        const int r0 = d.x;
        const bool window = d.y >= 0;
        const int clo = d.y, chi = d.z;
        const int r1 = window ? r0 + 1 : (u + 1 < nunits ? g.utab[u + 1].x : g.m);
        const int nrows = r1 - r0;
        if (tid == 0) L.nbig = 0;
        for (int i = tid; i <= nrows; i += FZ_WG) {
            L.rp[i] = g.rpA[r0 + i];
            L.rseg[i] = 0;
            L.rnnz[i] = 0;
        }
        {
            uint4 *k4 = reinterpret_cast<uint4 *>(L.keys);
            uint4 *i4 = reinterpret_cast<uint4 *>(L.info);
            for (int i = tid; i < FZ_H / 4; i += FZ_WG) {
                k4[i] = make_uint4(FZ_EMPTY, FZ_EMPTY, FZ_EMPTY, FZ_EMPTY);
                i4[i] = make_uint4(0u, 0u, 0u, 0u);
            }
        }
        __syncthreads();
        const int a0 = L.rp[0], a1 = L.rp[nrows];
        const long long prod = window ? (long long)d.w : g.cum[a1] - g.cum[a0];
        // ---- walk 1: segments + masks (+ product slot cache)
        fz_walk<false>(L, a0, a1, nrows, g.ebnd, g.Bcol, g.vA, window, clo, chi,
                       [&](int p, int b, int lr, double) {
                           const int c = g.Bcol[b];
                           const u32 key = ((u32)lr << 24) | (u32)(c >> 4);
                           u32 h = fz_hash(key);
                           while (true) {
                               const u32 k = L.keys[h];
                               if (k == key) break;
                               if (k == FZ_EMPTY) {
                                   const u32 old = atomicCAS(&L.keys[h], FZ_EMPTY, key);
                                   if (old == FZ_EMPTY) {
                                       const int idx = atomicAdd(&L.rseg[lr], 1);
                                       atomicOr(&L.info[h], (u32)idx << 16);
                                       break;
                                   }
                                   if (old == key) break;
                               }
                               h = (h + 1) & (FZ_H - 1);
                           }
                           atomicOr(&L.info[h], 1u << (c & 15));
                           if (p < FZ_PS) L.pslot[p] = (u16)(h | ((u32)(c & 15) << FZ_HBITS));
                       });
        FZ_PROF(1);
        // ---- rows: segment list offsets
        int S;
        {
            const int cnt = tid < nrows ? L.rseg[tid] : 0;
            const int ex = fz_excl_scan(cnt, &S, L.red);
            if (tid < nrows) {
                L.rseg[tid] = ex;
                if (cnt > FZ_SMALLROW) L.big[atomicAdd(&L.nbig, 1)] = tid;  // ordered by bitonic networks
            }
            if (tid == 0) L.rseg[nrows] = S;
        }
        __syncthreads();
        // ---- segment list + the unit's nnz (sum of the row masks' popcounts)
        int N;
        {
            int cn = 0;
            for (int h = tid; h < FZ_H; h += FZ_WG) {
                const u32 k = L.keys[h];
                if (k != FZ_EMPTY) {
                    const int lr = (int)(k >> 24);
                    const u32 inf = L.info[h];
                    L.v.sortv[L.rseg[lr] + (int)(inf >> 16)] = ((k & 0xffffffu) << 8) | (u32)lr;
                    cn += __popc(inf & 0xffffu);
                }
            }
            N = fz_sum(cn, L.red);
        }
        // ---- publish the aggregate; the predecessors' status loads fly during the ordering
        unsigned long long lb = 0;
        if (wave_id() == 0) lb = fz_publish(g.status, u, N);
        FZ_PROF(2);
        // ---- order each row's segments by tile column
        {
            u32 vv[FZ_SPT];
            int dst[FZ_SPT];
#pragma unroll
            for (int j = 0; j < FZ_SPT; ++j) {
                const int q = tid + j * FZ_WG;
                dst[j] = -1;
                if (q < S) {
                    const u32 v = L.v.sortv[q];
                    const int lr = (int)(v & 255u), ro = L.rseg[lr], n = L.rseg[lr + 1] - ro;
                    vv[j] = v;
                    if (n <= FZ_SMALLROW) {
                        int rank = 0;
                        for (int i = 0; i < n; ++i) rank += L.v.sortv[ro + i] < v ? 1 : 0;
                        dst[j] = ro + rank;
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < FZ_SPT; ++j)
                if (dst[j] >= 0) L.v.sortv[dst[j]] = vv[j];
            const int nbig = L.nbig;
            if (nbig) {
                // rows over FZ_SMALLROW segments: bitonic, a wave per row (<= 1024), else the workgroup
                for (int k = wave_id(); k < nbig; k += FZ_NW) {
                    const int lr = L.big[k], ro = L.rseg[lr], n = L.rseg[lr + 1] - ro;
                    if (n <= 1024) fz_bitonic<false>(L.v.sortv + ro, n);
                }
                __syncthreads();
                for (int k = 0; k < nbig; ++k) {  // uniform
                    const int lr = L.big[k], ro = L.rseg[lr], n = L.rseg[lr + 1] - ro;
                    if (n > 1024) fz_bitonic<true>(L.v.sortv + ro, n);
                }
            }
            __syncthreads();
        }
        FZ_PROF(3);
        // ---- segment offsets in CSR order: scan of mask popcounts over the sorted list
        {
            int hh[FZ_SPT], cc[FZ_SPT];
            int loc = 0;
            const int q0 = tid * FZ_SPT;
#pragma unroll
            for (int j = 0; j < FZ_SPT; ++j) {
                const int q = q0 + j;
                hh[j] = -1;
                cc[j] = 0;
                if (q < S) {
                    const u32 v = L.v.sortv[q];
                    const u32 key = ((v >> 8) & 0xffffffu) | ((v & 255u) << 24);
                    const int h = fz_probe(L.keys, key);
                    hh[j] = h;
                    cc[j] = __popc(L.info[h] & 0xffffu);
                    loc += cc[j];
                }
            }
            int tot;
            int off = fz_excl_scan(loc, &tot, L.red);
#pragma unroll
            for (int j = 0; j < FZ_SPT; ++j) {
                if (hh[j] >= 0) {
                    const u32 inf = L.info[hh[j]];
                    L.info[hh[j]] = ((u32)off << 16) | (inf & 0xffffu);
                    atomicAdd(&L.rnnz[L.keys[hh[j]] >> 24], cc[j]);
                    off += cc[j];
                }
            }
        }
        __syncthreads();
        my_seg += (tid == 0) ? S : 0;
        // rows: nonzero offsets in the unit's output
        {
            const int cnt = tid < nrows ? L.rnnz[tid] : 0;
            int tot;
            const int ex = fz_excl_scan(cnt, &tot, L.red);
            if (tid < nrows) L.rnnz[tid] = ex;
        }
        FZ_PROF(4);
        // ---- the unit's global CSR offset (look-back resolved; ticket order = row order)
        if (wave_id() == 0) {
            const long long e = fz_resolve(g.status, u, N, lb, g.overflow);
            if (lane_id() == 0) L.bc[0] = e;
        }
        __syncthreads();
        FZ_PROF(5);
        const long long E = L.bc[0];
        const bool fits = E + N <= g.cap;
        if (!fits && tid == 0) atomicExch(g.overflow, 1);
        if (fits) {
            if (!window || clo == 0)
                for (int i = tid; i < nrows; i += FZ_WG) g.Crp[r0 + i] = (int)(E + L.rnnz[i]);
            if (u == nunits - 1 && tid == 0) {
                g.Crp[g.m] = (int)(E + N);
                g.overflow[1] = (int)(E + N);  // nnz(C), read back with the flags
            }
            // columns, in sorted segment order
            for (int q = tid; q < S; q += FZ_WG) {
                const u32 v = L.v.sortv[q];
                const u32 key = ((v >> 8) & 0xffffffu) | ((v & 255u) << 24);
                const u32 inf = L.info[fz_probe(L.keys, key)];
                u32 msk = inf & 0xffffu;
                int o = (int)(inf >> 16);
                const int cb = (int)((v >> 8) & 0xffffffu) << 4;
                while (msk) {
                    g.Ccol[E + o++] = cb + __ffs(msk) - 1;
                    msk &= msk - 1;
                }
            }
        }
        __syncthreads();  // sortv (aliases vals) is dead from here
        FZ_PROF(6);
        const bool lds = N <= FZ_NV;
        if (lds) {
            for (int i = tid; i < N; i += FZ_WG) L.v.vals[i] = 0.0;
        } else if (fits) {
            for (int i = tid; i < N; i += FZ_WG) g.Cval[E + i] = 0.0;
        }
        __syncthreads();
        const bool cache = prod <= FZ_PS;
        // ---- walk 2: values at offset + popcount(mask below the column)
        if (fits || lds)
            fz_walk<true>(L, a0, a1, nrows, g.ebnd, g.Bcol, g.vA, window, clo, chi,
                          [&](int p, int b, int lr, double av) {
                              int h, cb;
                              if (cache) {
                                  const u32 ps = L.pslot[p];
                                  h = (int)(ps & (FZ_H - 1));
                                  cb = (int)(ps >> FZ_HBITS);
                              } else {
                                  const int c = g.Bcol[b];
                                  cb = c & 15;
                                  h = fz_probe(L.keys, ((u32)lr << 24) | (u32)(c >> 4));
                              }
                              const u32 inf = L.info[h];
                              const int pos = (int)(inf >> 16) + __popc(inf & ((1u << cb) - 1u));
                              const double x = av * g.Bval[b];
                              if (lds) atomicAdd(&L.v.vals[pos], x);
                              else unsafeAtomicAdd(&g.Cval[E + pos], x);
                          });
        FZ_PROF(7);
        if (lds && fits)
            for (int i = tid; i < N; i += FZ_WG) g.Cval[E + i] = L.v.vals[i];
        __syncthreads();
        FZ_PROF(8);
    }
    if (tid == 0 && my_seg) atomicAdd(g.nseg, (unsigned long long)my_seg);
#ifdef TSG_FZ_PROF
    if (tid == 0)
        for (int k = 0; k < 9; ++k) atomicAdd(&g.prof[k], prof_acc[k]);
#endif
}

// ---------------------------------------------------------------------------
// routing statistic: the longest row of a CSR (read back with the sortedness
// flag; the fused path takes products whose rows are short on both sides)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_fz_maxlen(const int *rp, int m, int *out) {
    __shared__ int red[2 * WAVES];
    int mx = 0, mn = 0;
    for (int r = blockIdx.x * WG + threadIdx.x; r < m; r += gridDim.x * WG) mx = max(mx, rp[r + 1] - rp[r]);
    block_minmax(mn, mx, red);  // one atomic per workgroup
    if (threadIdx.x == 0 && mx > 0) atomicMax(out, mx);
}

int dev_row_maxlen_async(Context &cx, const tsg_dev_csr &M, int *host_out, hipStream_t s) {
    int *d = nullptr;
    TSG_TRY(cx.get(&d, 1));
    TSG_HIP(hipMemsetAsync(d, 0, sizeof(int), s));
    if (M.m > 0) k_fz_maxlen<<<grid_for(M.m, WG * 8, 512), WG, 0, s>>>(M.rowpointer, M.m, d);
    TSG_HIP(hipGetLastError());
    TSG_HIP(hipMemcpyAsync(host_out, d, sizeof(int), hipMemcpyDeviceToHost, s));
    cx.put(d);
    return TSG_OK;
}

// ---------------------------------------------------------------------------
// host orchestration: CSR in -> CSR out
// ev (optional, >= 6 events): 0 start | 1 units built | 4..5 the unit kernel | 3 end
// ---------------------------------------------------------------------------
int dev_spgemm_fused(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, tsg_dev_csr &C, tsg_stats *st,
                     hipStream_t s, hipEvent_t *ev, int2 *ebnd_pre, long long *cum_pre) {
    if (A.n != B.m) return TSG_ERR_INVALID;
    const int m = A.m;
    const long nnzA = A.nnz;
    if ((long long)B.n >= kFusedMaxCols) return TSG_ERR_UNSUPPORTED;  // tile column < 2^24 in a segment key
    C = tsg_dev_csr{};
    C.m = m;
    C.n = B.n;
    if (ev && !(ebnd_pre && cum_pre)) TSG_HIP(hipEventRecord(ev[0], s));  // (else the caller's, before the shared setup)
    int2 *ebnd = nullptr;
    long long *cum = nullptr;
    int *ucnt = nullptr, *hlist = nullptr, *ctr = nullptr, *wofs = nullptr;
    const bool pre = ebnd_pre && cum_pre;
    if (pre) {
        ebnd = ebnd_pre;
        cum = cum_pre;
    } else {
        TSG_TRY(cx.get(&ebnd, (size_t)nnzA + 1));
        TSG_TRY(cx.get(&cum, (size_t)nnzA + 1));
    }
    TSG_TRY(cx.get(&ucnt, (size_t)m + 1));
    TSG_TRY(cx.get(&hlist, (size_t)m + 1));
    TSG_TRY(cx.get(&wofs, (size_t)m + 1));
    // ctr (ints): [0] heavy rows [2..3] heavy products [4] window top [5] ticket [6] overflow
    //            [7] nnz(C) [8..9] products [10..11] C row-segments
    TSG_TRY(cx.get(&ctr, 16));
    TSG_HIP(hipMemsetAsync(ctr, 0, 16 * sizeof(int), s));
    if (!pre) {
        k_fz_entries<<<grid_for(nnzA + 1, WG, 16384), WG, 0, s>>>(A.columnindex, nnzA, B.rowpointer, ebnd, cum);
        TSG_HIP(hipGetLastError());
        TSG_TRY(scan_exclusive_i64(cx, cum, nnzA + 1, s));
    }
    k_fz_rows<<<grid_for(((long)m + FZ_ROWS - 1) / FZ_ROWS, WAVES, 4096), WG, 0, s>>>(A.rowpointer, m, cum, nnzA,
                                                                                   ucnt, hlist, ctr);
    TSG_HIP(hipGetLastError());
    // one host round trip: the product total (output bound) and the heavy rows
    TSG_HIP(hipMemcpyAsync(cx.pinned64, ctr, 12 * sizeof(int), hipMemcpyDeviceToHost, s));
    TSG_TRY(stream_wait(s));
    const int nheavy = reinterpret_cast<const int *>(cx.pinned64)[0];
    const unsigned long long heavyP = reinterpret_cast<const unsigned long long *>(cx.pinned64)[1];
    const long long total = cx.pinned64[4];
    if (nheavy > 0) TSG_HIP(hipMemsetAsync(wofs, 0xff, ((size_t)m + 1) * sizeof(int), s));
    int binw = 2048, nbins = 0;
    if ((long long)B.n > (long long)FZ_MAXBINS * 2048) binw = (int)((((long long)B.n + FZ_MAXBINS - 1) / FZ_MAXBINS + 15) / 16 * 16);
    nbins = (int)(((long long)B.n + binw - 1) / binw);
    const long long wcap = nheavy ? 3 * (long long)(heavyP / (FZ_CAP / 2)) + 2LL * nheavy + 1 : 1;
    int4 *wtab = nullptr;
    int *wtop = ctr + 4;
    TSG_TRY(cx.get(&wtab, (size_t)wcap));
    if (nheavy > 0)
        k_fz_heavy<<<grid_for(nheavy, 1, 4096), WG, 0, s>>>(hlist, ctr, A.rowpointer, ebnd, B.columnindex, B.n,
                                                             binw, nbins, ucnt, wofs, wtab, wtop);
    TSG_HIP(hipGetLastError());
    TSG_TRY(scan_exclusive_i32(cx, ucnt, (long)m + 1, s));  // ucnt -> unit base per row; [m] = #units
    const long long maxu = (long long)m + wcap + 1;
    int4 *utab = nullptr;
    unsigned long long *status = nullptr;
    unsigned long long *nseg = reinterpret_cast<unsigned long long *>(ctr + 10);
    TSG_TRY(cx.get(&utab, (size_t)maxu));
    TSG_TRY(cx.get(&status, (size_t)maxu + 12));
    int *ticket = ctr + 5, *overflow = ctr + 6;
    TSG_HIP(hipMemsetAsync(status, 0, ((size_t)maxu + 12) * sizeof(unsigned long long), s));
    if (m > 0)
        k_fz_fill<<<grid_for(m, WG, 16384), WG, 0, s>>>(ucnt, m, nheavy ? wofs : nullptr, wtab, utab);
    TSG_HIP(hipGetLastError());
    if (ev) TSG_HIP(hipEventRecord(ev[1], s));
    const long long cap = total < 0x7fffffffLL ? total : 0x7fffffffLL;
    TSG_TRY(cx.get(&C.rowpointer, (size_t)m + 1));
    TSG_TRY(cx.get(&C.columnindex, (size_t)cap + 1));
    TSG_TRY(cx.get(&C.value, (size_t)cap + 1));
    if (m == 0) TSG_HIP(hipMemsetAsync(C.rowpointer, 0, sizeof(int), s));
    if (ev) TSG_HIP(hipEventRecord(ev[4], s));
    if (m > 0) {
        FzArgs g{A.rowpointer, A.columnindex, A.value, ebnd, cum, B.columnindex, B.value, utab, ucnt + m, m, cap,
                 status, ticket, C.rowpointer, C.columnindex, C.value, overflow, nseg, status + maxu + 1};
        k_fz_units<<<512, FZ_WG, 0, s>>>(g);
        TSG_HIP(hipGetLastError());
    }
    if (ev) TSG_HIP(hipEventRecord(ev[5], s));
    // the one read-back after the kernel: nnz(C), the overflow flag, the segment count
    TSG_HIP(hipMemcpyAsync(cx.pinned64, ctr, 12 * sizeof(int), hipMemcpyDeviceToHost, s));
    if (ev) TSG_HIP(hipEventRecord(ev[3], s));
    TSG_TRY(stream_wait(s));
#ifdef TSG_FZ_PROF
    {
        unsigned long long pr[9];
        TSG_HIP(hipMemcpy(pr, status + maxu + 1, sizeof(pr), hipMemcpyDeviceToHost));
        double tot = 0;
        for (unsigned long long x : pr) tot += (double)x;
        static const char *nm[9] = {"ticket", "setup+walk1", "list", "order", "offsets", "lookback", "columns",
                                    "walk2", "values"};
        fprintf(stderr, "k_fz_units phases (%% of workgroup time):");
        for (int k = 0; k < 9; ++k) fprintf(stderr, " %s %.1f", nm[k], 100.0 * (double)pr[k] / tot);
        fprintf(stderr, "  (total %.3g ticks)\n", tot);
    }
#endif
    if (!pre) {
        cx.put(ebnd);
        cx.put(cum);
    }
    cx.put(ucnt);
    cx.put(hlist);
    cx.put(wofs);
    cx.put(ctr);
    cx.put(wtab);
    cx.put(utab);
    cx.put(status);
    const int *pc = reinterpret_cast<const int *>(cx.pinned64);
    if (pc[6] == 2) return TSG_ERR_HIP;  // look-back stalled (never expected)
    if (pc[6]) return TSG_ERR_OVERFLOW;
    C.nnz = m > 0 ? pc[7] : 0;
    if (st) {
        st->nnzC = C.nnz;
        st->tile_products = total;
        st->numblkC = cx.pinned64[5];  // C row-segments (see tsg.h)
    }
    return TSG_OK;
}

}  // namespace tsg
