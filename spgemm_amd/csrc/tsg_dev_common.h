// tsg_dev_common.h -- wave64 / workgroup primitives shared by the gfx950 kernels
// (tsg_device.hip: csr2tile, the tiled steps, tile2csr; tsg_rows.hip, tsg_band.hip:
// the row-merge and banded CSR paths).  Device code only; include after tsg_internal.h.
#pragma once

#include <climits>

#include "tsg_internal.h"

namespace tsg {

typedef unsigned long long u64;
typedef unsigned int u32;
typedef unsigned short u16;

constexpr int WG = 256;
constexpr int WAVES = WG / 64;

// ---------------------------------------------------------------------------
// wave / workgroup primitives
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 32-bit inclusive wave scans on DPP lane moves (no LDS permute round trips):
// row_shr 1/2/4/8 scan each 16-lane row, row_bcast:15 / :31 carry the row
// totals into rows 1, 3 and 2, 3.  id = the operator's identity (what lanes
// without a source read).  The whole wave must be active.
template <int CTRL, int RM> __device__ __forceinline__ int dpp_mov(int id, int v) {
    return __builtin_amdgcn_update_dpp(id, v, CTRL, RM, 0xf, false);
}
template <class Op> __device__ __forceinline__ int wave_incl_dpp(int v, int id, Op op) {
    v = op(v, dpp_mov<0x111, 0xf>(id, v));  // row_shr:1
    v = op(v, dpp_mov<0x112, 0xf>(id, v));  // row_shr:2
    v = op(v, dpp_mov<0x114, 0xf>(id, v));  // row_shr:4
    v = op(v, dpp_mov<0x118, 0xf>(id, v));  // row_shr:8
    v = op(v, dpp_mov<0x142, 0xa>(id, v));  // row_bcast:15
    v = op(v, dpp_mov<0x143, 0xc>(id, v));  // row_bcast:31
    return v;
}
struct OpAdd {
    __device__ int operator()(int a, int b) const { return a + b; }
};
struct OpMin {
    __device__ int operator()(int a, int b) const { return min(a, b); }
};
struct OpMax {
    __device__ int operator()(int a, int b) const { return max(a, b); }
};
__device__ __forceinline__ int wave_incl_scan_dpp(int v) { return wave_incl_dpp(v, 0, OpAdd{}); }

template <class T> __device__ __forceinline__ T wave_incl_scan(T x) {
    if constexpr (sizeof(T) == 4) {
        return (T)wave_incl_scan_dpp((int)x);
    } else {
        const int l = lane_id();
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            T y = __shfl_up(x, d, 64);
            if (l >= d) x += y;
        }
        return x;
    }
}

__device__ __forceinline__ int wave_incl_max(int x) { return wave_incl_dpp(x, INT_MIN, OpMax{}); }

// the value of lane 63 (a scan's total), as a wave-uniform value
__device__ __forceinline__ int wave_last(int x) { return __builtin_amdgcn_readlane(x, 63); }

template <class T> __device__ __forceinline__ T wave_sum(T x) {
    if constexpr (sizeof(T) == 4) {
        return (T)wave_last(wave_incl_scan_dpp((int)x));
    } else {
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
        return x;
    }
}

// exclusive scan across the 256-thread workgroup; red needs WAVES entries
template <class T> __device__ __forceinline__ T block_excl_scan(T x, T *total, T *red) {
    const T inc = wave_incl_scan(x);
    if (lane_id() == 63) red[wave_id()] = inc;
    __syncthreads();
    T off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
        T v = red[w];
        off += (w < wave_id()) ? v : T(0);
        tot += v;
    }
    __syncthreads();
    *total = tot;
    return off + inc - x;
}

// workgroup min and max of x (red: 2*WAVES ints)
__device__ __forceinline__ void block_minmax(int &mn, int &mx, int *red) {
    mn = wave_last(wave_incl_dpp(mn, INT_MAX, OpMin{}));
    mx = wave_last(wave_incl_dpp(mx, INT_MIN, OpMax{}));
    if (lane_id() == 0) {
        red[wave_id()] = mn;
        red[WAVES + wave_id()] = mx;
    }
    __syncthreads();
    mn = red[0];
    mx = red[WAVES];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) {
        mn = min(mn, red[w]);
        mx = max(mx, red[WAVES + w]);
    }
    __syncthreads();
}

template <class T> __device__ __forceinline__ T block_sum(T x, T *red) {
    x = wave_sum(x);
    if (lane_id() == 0) red[wave_id()] = x;
    __syncthreads();
    T tot = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) tot += red[w];
    __syncthreads();
    return tot;
}

// first index in [lo,hi) with a[idx] >= key
template <class T>
__device__ __forceinline__ int lower_bound_dev(const T *a, int lo, int hi, T key) {
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Branchless lower bound for WAVE-UNIFORM bounds: the trip count depends only
// on the (uniform) range length, so the loop has no exec-mask bookkeeping and
// the body is compare + select around one LDS read.
// first index in [lo,hi) with a[idx] >= key
__device__ __forceinline__ int lower_bound_u(const int *a, int lo, int hi, int key) {
    int len = hi - lo, base = lo;
    if (len <= 0) return lo;
    while (len > 1) {
        const int half = len >> 1;
        base = (a[base + half - 1] < key) ? base + half : base;
        len -= half;
    }
    return base + (a[base] < key ? 1 : 0);
}
// largest l in [0, n) with off[l] <= it (off non-decreasing, off[0] <= it).
// A branchless fixed-step variant measured slower here.
__device__ __forceinline__ int owner_search(const int *off, int n, int it) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= it) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// XCD-aware work order: the dispatcher deals a grid's workgroups round-robin
// over the 8 XCDs (workgroup b to XCD b % 8), each with its own L2.  This maps
// workgroup b to item xcd_item(b, n) of n so that every XCD takes one
// contiguous range of items, in order: neighbouring rows (which read
// neighbouring B rows in banded and local web-graph operands) share an L2.
constexpr int kXcds = 8;
__device__ __forceinline__ int xcd_item(int b, int n) {
    const int q = n / kXcds, r = n % kXcds, x = b % kXcds, k = b / kXcds;
    return x * q + min(x, r) + k;
}

static inline int grid_for(long work, int per_block, int cap) {
    long g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}


}  // namespace tsg
