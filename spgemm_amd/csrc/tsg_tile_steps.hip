// tsg_tile_steps.hip -- steps 2 and 3 of TileSpGEMM on the reference's tiled
// layout at any tile size tm x tn (tm, tn in {16, 32, 48, 64}), for the host
// tile API (tsg_tilespgemm, the ./test CLI path).  gfx950, wave64.
//
// Reference (paths under /root/reference/src):
//   step 2  tilespgemm-cuda.h:394-773   per C tile: intersect A's tile row i with
//           B's tile column j (binary search of each A tile in B's column,
//           intersection_binarysearch_kernel :167-211), OR the B tile rows'
//           masks into C's row masks for every A nonzero, popcount -> tile nnz
//           and row pointers
//   scan    :2598-2604                   exclusive scan of the tile nnz
//   step 3  :1273-2218                   per C tile: values with the adaptive
//           accumulator -- sparse (rank of the column in the row mask) for
//           tiles of <= 512 nonzeros, dense (tm x tm) above, the
//           reference's dns / ful bins (without its shared global scratch,
//           :1980, :2625-2626: here each group owns its accumulator in LDS)
//
// 64 / tm C tiles per wave (16: four, 32: two, 48 and 64: one), a group of tm
// lanes per tile.  Lane r of a group owns row r of its tile: its row mask lives
// in one 64-bit register (column c = bit c), its row pointer comes from a group
// scan of the popcounts, and in step 3 it accumulates only its own row's
// entries, so the accumulator needs no atomics.  The matched (A tile, B tile)
// pairs: the group's lanes take tm A tiles of row i at a time, each binary-
// searches B's tile column j, and the matches (a ballot, ascending k) are
// visited in order.
#include "tsg_internal.h"
#include "tsg_dev_common.h"

namespace tsg {

namespace {

constexpr int TS_SPARSE_MAX = 512;  // tiles up to this many nonzeros: sparse accumulator

struct TileArgs {
    // A: row-major tiles (tm x tn), Col encoded r * tn + c
    const int *Aptr, *Acol, *Annz;
    const u16 *APtr, *ACol;
    const double *AVal;
    // B: CSC tile order (tn x tm tiles), Col = local column, masks tm/16 words per row
    const int *Bcptr, *Browidx, *Bnnz;
    const u16 *BPtr, *BCol, *Bmask;
    const double *BVal;
    // C (tm x tm tiles): step-1 structure + outputs
    const int *Crow, *Ccol;
    int numtile, tn;
    int *Cnnz;
    u16 *CPtr, *Cmask, *CCol;
    double *CVal;
};

// the reference's u16 mask words (bit 15 - c%16 of word c/16) <-> column bits of a u64
template <int TM> __device__ __forceinline__ unsigned long long row_bits(const u16 *w) {
    unsigned long long m = 0;
#pragma unroll
    for (int k = 0; k < TM / 16; ++k) m |= (unsigned long long)(__brev((u32)w[k]) >> 16) << (16 * k);
    return m;
}
template <int TM> __device__ __forceinline__ void store_row_bits(u16 *w, unsigned long long m) {
#pragma unroll
    for (int k = 0; k < TM / 16; ++k) w[k] = (u16)(__brev((u32)((m >> (16 * k)) & 0xffffu)) >> 16);
}

// every matched (A tile a, B tile q) of the group's C tile (i, j), in ascending k:
// f(a, q) on every lane of the group (live: the group has a tile; the loop runs
// until every group of the wave is done -- no wave-level barrier inside)
template <int TM, class F>
__device__ __forceinline__ void for_each_match(const TileArgs &g, bool live, int i, int j, int gbase, int gl,
                                               F &&f) {
    const unsigned long long gmask = (TM == 64 ? ~0ull : ((1ull << TM) - 1ull)) << gbase;
    int pa = live ? g.Aptr[i] : 0;
    const int ea = live ? g.Aptr[i + 1] : 0;
    const int pb = live ? g.Bcptr[j] : 0, eb = live ? g.Bcptr[j + 1] : 0;
    for (;; pa += TM) {
        if (!__any(pa < ea)) break;  // (wave-uniform)
        const int a = pa + gl;
        int q = -1;
        if (a < ea) {
            const int k = g.Acol[a];
            const int lo = lower_bound_dev(g.Browidx, pb, eb, k);
            q = lo < eb && g.Browidx[lo] == k ? lo : -1;
        }
        unsigned long long mm = __ballot(q >= 0) & gmask;
        while (__any(mm != 0)) {  // (the groups' match counts differ: idle groups wait)
            const int src = mm ? (int)__builtin_ctzll(mm) : 0;
            const int am = __shfl(a, src, 64), qm = __shfl(q, src, 64);
            if (mm) {
                mm &= mm - 1ull;
                f(am, qm);
            }
        }
    }
}

// A tile a, row r: its entries [s, e) (absolute positions)
template <int TM> __device__ __forceinline__ void a_row(const TileArgs &g, int a, int r, int &s, int &e) {
    const int base = g.Annz[a];
    s = base + g.APtr[(size_t)a * TM + r];
    e = r + 1 < TM ? base + g.APtr[(size_t)a * TM + r + 1] : g.Annz[a + 1];
}

// inclusive scan of v over the tm lanes of each group (groups of 16, 32, 48 or 64)
template <int TM> __device__ __forceinline__ int group_incl_scan(int v, int gl) {
#pragma unroll
    for (int d = 1; d < TM; d <<= 1) {
        const int y = __shfl_up(v, d, 64);
        if (gl >= d) v += y;
    }
    return v;
}

}  // namespace

template <int TM> __global__ __launch_bounds__(WG) void k_tile_step2(TileArgs g) {
    constexpr int G = 64 / TM;  // C tiles per wave
    const int lane = lane_id(), grp = lane / TM, gl = lane - grp * TM, gbase = grp * TM;
    const long nwaves = ((long)gridDim.x * WG) >> 6;
    for (long t0 = (((long)blockIdx.x * WG + threadIdx.x) >> 6) * G; t0 < g.numtile; t0 += nwaves * G) {
        const long t = t0 + grp;
        const bool live = grp < G && t < g.numtile;
        const int i = live ? g.Crow[t] : 0, j = live ? g.Ccol[t] : 0;
        unsigned long long msk = 0;
        for_each_match<TM>(g, live, i, j, gbase, gl, [&](int a, int q) {
            int s, e;
            a_row<TM>(g, a, gl, s, e);
            for (int x = s; x < e; ++x) {
                const int c = (int)g.ACol[x] - gl * g.tn;  // A's Col = r * tn + c
                msk |= row_bits<TM>(g.Bmask + ((size_t)q * g.tn + c) * (TM / 16));
            }
        });
        const int cnt = live ? __popcll(msk) : 0;
        const int inc = group_incl_scan<TM>(cnt, gl);
        const int nnz = __shfl(inc, gbase + TM - 1, 64);
        if (live) {
            g.CPtr[(size_t)t * TM + gl] = (u16)(inc - cnt);
            store_row_bits<TM>(g.Cmask + ((size_t)t * TM + gl) * (TM / 16), msk);
            if (gl == 0) g.Cnnz[t] = nnz;
        }
    }
}

// step 3: one wave per workgroup (the dense accumulator of a 64 x 64 tile is
// 32 KB of LDS); a group's accumulator: its tile's nonzeros (sparse: the rank
// of the column in the row) or tm x tm (dense)
template <int TM> constexpr int s3_slots() {
    return (64 / TM) * TS_SPARSE_MAX > TM * TM ? (64 / TM) * TS_SPARSE_MAX : TM * TM;
}
template <int TM> __global__ __launch_bounds__(64) void k_tile_step3(TileArgs g) {
    constexpr int G = 64 / TM;
    __shared__ double acc[s3_slots<TM>()];
    const int lane = lane_id(), grp = lane / TM, gl = lane - grp * TM, gbase = grp * TM;
    for (long t0 = (long)blockIdx.x * G; t0 < g.numtile; t0 += (long)gridDim.x * G) {
        const long t = t0 + grp;
        bool live = grp < G && t < g.numtile;
        const int off = live ? g.Cnnz[t] : 0, nnz = live ? g.Cnnz[t + 1] - off : 0;
        live = live && nnz > 0;
        // a dense tile takes the whole accumulator: the wave's groups run it alone
        const bool dense_any = __any(live && nnz > TS_SPARSE_MAX);
        for (int pass = 0; pass < (dense_any ? G : 1); ++pass) {  // (wave-uniform)
            const bool mine = live && (!dense_any || grp == pass);
            const bool dense = nnz > TS_SPARSE_MAX;
            double *A = acc + (dense_any ? 0 : grp * TS_SPARSE_MAX);
            const int i = mine ? g.Crow[t] : 0, j = mine ? g.Ccol[t] : 0;
            unsigned long long msk = 0;
            int rp = 0;
            if (mine) {
                msk = row_bits<TM>(g.Cmask + ((size_t)t * TM + gl) * (TM / 16));
                rp = g.CPtr[(size_t)t * TM + gl];
            }
            const int span = mine ? (dense ? TM * TM : nnz) : 0;
            for (int k = gl; k < span; k += TM) A[k] = 0.0;
            wave_lds_sync();
            for_each_match<TM>(g, mine, i, j, gbase, gl, [&](int a, int q) {
                int s, e;
                a_row<TM>(g, a, gl, s, e);
                const int bbase = g.Bnnz[q];
                for (int x = s; x < e; ++x) {
                    const int c = (int)g.ACol[x] - gl * g.tn;
                    const double va = g.AVal[x];
                    const int bs = bbase + g.BPtr[(size_t)q * g.tn + c];
                    const int be = c + 1 < g.tn ? bbase + g.BPtr[(size_t)q * g.tn + c + 1] : g.Bnnz[q + 1];
                    for (int y = bs; y < be; ++y) {
                        const int cb = g.BCol[y];
                        const int slot = dense ? gl * TM + cb : rp + __popcll(msk & ((1ull << cb) - 1ull));
                        A[slot] += va * g.BVal[y];  // lane-private row: no atomics
                    }
                }
            });
            wave_lds_sync();
            if (mine) {
                unsigned long long m = msk;
                int k = off + rp, rank = rp;
                while (m) {
                    const int c = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    g.CCol[k] = (u16)c;
                    g.CVal[k] = dense ? A[gl * TM + c] : A[rank];
                    ++k;
                    ++rank;
                }
            }
            wave_lds_sync();
        }
    }
}

// tile_rowidx: a wave per tile row, its lanes over the row's tiles (coalesced)
__global__ __launch_bounds__(WG) void k_tile_crow(const int *Cptr, int tilem, int *Crow) {
    const int lane = lane_id();
    for (int i = (blockIdx.x * WG + threadIdx.x) >> 6; i < tilem; i += (gridDim.x * WG) >> 6)
        for (int t = Cptr[i] + lane; t < Cptr[i + 1]; t += 64) Crow[t] = i;
}


// Steps 2 and 3 at tile size C.tile_m x C.tile_m on the step-1 structure already
// in C (tile_ptr, tile_columnidx, numtile): fills tile_rowidx, tile_nnz
// (exclusive, numtile + 1), tile_csr_Ptr, mask, tile_csr_Col, tile_csr_Value,
// nnz.  ev (optional): records ev[1] before step 2, ev[2] after the scan,
// ev[3] after step 3.
int dev_tile_steps23(Context &cx, const tsg_dev_tiles &A, const tsg_dev_tiles &B, tsg_dev_tiles &C, hipStream_t s,
                     hipEvent_t *ev) {
    const int tm = C.tile_m, tn = A.tile_n;
    if (!(tm == 16 || tm == 32 || tm == 48 || tm == 64) || A.tile_m != tm || B.tile_m != tn || B.tile_n != tm)
        return TSG_ERR_UNSUPPORTED;
    if (!B.csc_tile_ptr || !B.csc_tile_rowidx || !B.mask) return TSG_ERR_INVALID;
    const int nt = C.numtile;
    TSG_TRY(cx.get(&C.tile_rowidx, (size_t)nt + 1));
    TSG_TRY(cx.get(&C.tile_nnz, (size_t)nt + 1));
    TSG_TRY(cx.get(&C.tile_csr_Ptr, (size_t)nt * tm + 1));
    TSG_TRY(cx.get(&C.mask, (size_t)nt * tm * (tm / 16) + 1));
    if (C.tilem > 0) k_tile_crow<<<grid_for(C.tilem, WAVES, 8192), WG, 0, s>>>(C.tile_ptr, C.tilem, C.tile_rowidx);
    TSG_HIP(hipMemsetAsync(C.tile_nnz + nt, 0, sizeof(int), s));
    TSG_HIP(hipGetLastError());
    TileArgs g{A.tile_ptr, A.tile_columnidx, A.tile_nnz, A.tile_csr_Ptr, A.tile_csr_Col, A.tile_csr_Value,
               B.csc_tile_ptr, B.csc_tile_rowidx, B.tile_nnz, B.tile_csr_Ptr, B.tile_csr_Col, B.mask,
               B.tile_csr_Value, C.tile_rowidx, C.tile_columnidx, nt, tn, C.tile_nnz, C.tile_csr_Ptr, C.mask,
               nullptr, nullptr};
    if (ev) TSG_HIP(hipEventRecord(ev[1], s));
    const int per_wave = 64 / tm;  // C tiles per wave
    const int grid = grid_for(((long)nt + per_wave - 1) / per_wave, WAVES, 65536);
    const int grid3 = grid_for(((long)nt + per_wave - 1) / per_wave, 1, 262144);  // (one wave per workgroup)
    if (nt > 0) {
        switch (tm) {
            case 16: k_tile_step2<16><<<grid, WG, 0, s>>>(g); break;
            case 32: k_tile_step2<32><<<grid, WG, 0, s>>>(g); break;
            case 48: k_tile_step2<48><<<grid, WG, 0, s>>>(g); break;
            default: k_tile_step2<64><<<grid, WG, 0, s>>>(g); break;
        }
    }
    TSG_HIP(hipGetLastError());
    long long nnz = 0;
    TSG_TRY(scan_exclusive_i32_total(cx, C.tile_nnz, (long)nt + 1, s, &nnz));
    C.nnz = (int)nnz;
    if (ev) TSG_HIP(hipEventRecord(ev[2], s));
    TSG_TRY(cx.get(&C.tile_csr_Col, (size_t)nnz + 1));
    TSG_TRY(cx.get(&C.tile_csr_Value, (size_t)nnz + 1));
    g.CCol = C.tile_csr_Col;
    g.CVal = C.tile_csr_Value;
    if (nt > 0 && nnz > 0) {
        switch (tm) {
            case 16: k_tile_step3<16><<<grid3, 64, 0, s>>>(g); break;
            case 32: k_tile_step3<32><<<grid3, 64, 0, s>>>(g); break;
            case 48: k_tile_step3<48><<<grid3, 64, 0, s>>>(g); break;
            default: k_tile_step3<64><<<grid3, 64, 0, s>>>(g); break;
        }
    }
    TSG_HIP(hipGetLastError());
    if (ev) TSG_HIP(hipEventRecord(ev[3], s));
    return TSG_OK;
}

}  // namespace tsg
