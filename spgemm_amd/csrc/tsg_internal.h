// tsg_internal.h -- host-side internals shared by the device code (tsg_device.hip)
// and the C-ABI layer (tsg_api.cpp).  gfx950 / wave64 only.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <unordered_map>
#include <vector>

#include "../../include/tsg.h"

namespace tsg {

#define TSG_HIP(call)                                                    \
    do {                                                                 \
        hipError_t _e = (call);                                          \
        if (_e != hipSuccess) {                                          \
            ::tsg::report_hip_error(_e, #call, __FILE__, __LINE__);      \
            return (_e == hipErrorOutOfMemory) ? TSG_ERR_OOM : TSG_ERR_HIP; \
        }                                                                \
    } while (0)

#define TSG_TRY(call)                   \
    do {                                \
        int _rc = (call);               \
        if (_rc != TSG_OK) return _rc;  \
    } while (0)

void report_hip_error(hipError_t e, const char *what, const char *file, int line);

// Wait for the stream's work: poll for up to ~1 ms (a blocking wait costs
// 20-50 us of wake-up on every mid-pipeline size read-back), then block.
int stream_wait(hipStream_t s);

// Caching device allocator: power-of-two size classes, blocks return to a free
// list and are reused by later allocations on the (single) call stream, so the
// steady-state pipeline performs no hipMalloc.
class DevicePool {
  public:
    ~DevicePool();
    int alloc(void **p, size_t bytes);
    void release(void *p);
    void release_all_live();  // returns every live block to the cache
    void trim();              // hipFree of the cached blocks
    size_t bytes_reserved() const { return reserved_; }

  private:
    std::multimap<size_t, void *> free_;
    std::unordered_map<void *, size_t> live_;
    size_t reserved_ = 0;
};

struct Context {
    int device = 0;
    DevicePool pool;
    int *pinned = nullptr;        // host pinned scratch for size read-backs
    long long *pinned64 = nullptr;
    int *dpinned = nullptr;        // device views of the pinned scratch (kernels report
    long long *dpinned64 = nullptr; //   small results there by system-scope stores)
    hipEvent_t ev[16];
    bool stage_ev = false;         // the stage events too (TSG_STAGE_EVENTS=1), not just the kernel bracket
    bool ev_ready = false;
    std::vector<void *> owned;    // outputs handed to the caller (released on reset)
    int init(int dev);
    void destroy();
    template <class T> int get(T **p, size_t count) {
        void *v = nullptr;
        int rc = pool.alloc(&v, count * sizeof(T) + 16);
        *p = static_cast<T *>(v);
        return rc;
    }
    void put(void *p) { if (p) pool.release(p); }
};

// ---- launchers implemented in tsg_device.hip (all stream-ordered, no sync) ----
// Exclusive scan in place over n elements (a[n-1] ends up = sum of a[0..n-2]
// when the caller stored 0 there, i.e. the reference's "n+1 scan" idiom).
int scan_exclusive_i32(Context &cx, int *a, long n, hipStream_t s);
int scan_exclusive_i64(Context &cx, long long *a, long n, hipStream_t s);
// Sort u64 keys ascending inside each segment [seg[i], seg[i+1]) in place.
int segmented_sort_u64(Context &cx, unsigned long long *keys, const int *seg, int nseg,
                       long total, hipStream_t s);

int launch_nnzcub(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B,
                  unsigned long long *d_out, hipStream_t s);
int dev_transpose(Context &cx, const tsg_dev_csr &A, tsg_dev_csr &out, hipStream_t s);
int dev_csr2tile_row_major(Context &cx, const tsg_dev_csr &A, int tm, int tn, tsg_dev_tiles &out,
                           hipStream_t s);
int dev_csr2tile_col_major(Context &cx, const tsg_dev_csr &B, int tm, int tn, tsg_dev_tiles &out,
                           hipStream_t s);
// csr_out != nullptr: step 3 also scatters C into CSR (tile2csr fused into its epilogue).
// Acsr/Bcsr (nullable; B's rows column-sorted): the CSR operands, enabling the
// element-streaming passes -- step 3's values always, step 2's masks when
// step2_elem.  A and B then only need their tile structure (tile_ptr,
// tile_columnidx) unless some step still reads the tile payloads.
int dev_tilespgemm(Context &cx, const tsg_dev_tiles &A, const tsg_dev_tiles &B, tsg_dev_tiles &C,
                   tsg_stats *st, hipStream_t s, hipEvent_t *ev_marks, tsg_dev_csr *csr_out,
                   const tsg_dev_csr *Acsr = nullptr, const tsg_dev_csr *Bcsr = nullptr,
                   bool step2_elem = false);
// step 1 alone: C tile structure (tile_ptr, tile_columnidx, numtile) of any tile size
int dev_step1(Context &cx, const tsg_dev_tiles &A, const tsg_dev_tiles &B, tsg_dev_tiles &C,
              long long *tile_products, hipStream_t s, const tsg_dev_csr *Ael = nullptr,
              const tsg_dev_csr *Bel = nullptr, int2 *ebnd = nullptr,
              long long **tbase_out = nullptr, long long *tslots_out = nullptr, bool fill_ebnd = false);
// the reference's tiled C payload (tile_nnz, Ptr, mask, Col, Value) laid onto
// step 1's 16 x 16 structure from a column-sorted CSR C (tsg_ctiles.hip)
int dev_ctiles_from_csr(Context &cx, const tsg_dev_csr &Cc, tsg_dev_tiles &C, hipStream_t s);
// steps 2 + 3 on the reference tiled layout at any tile size (tsg_tile_steps.hip):
// C holds step 1's structure at C.tile_m x C.tile_m; ev (optional) gets ev[1..3]
int dev_tile_steps23(Context &cx, const tsg_dev_tiles &A, const tsg_dev_tiles &B, tsg_dev_tiles &C, hipStream_t s,
                     hipEvent_t *ev);
// tile_ptr + tile_columnidx of a CSR's tiling (tr x tc tiles), no payload;
// tile_columnidx is left null when M.nnz < skip_emit_density * numtile
int dev_tile_structure(Context &cx, const tsg_dev_csr &M, int tr, int tc, tsg_dev_tiles &out, hipStream_t s,
                       double skip_emit_density = 0);
// row masks of a tiling (structure in t) straight from CSR, into a new zeroed array
int dev_tile_masks(Context &cx, const tsg_dev_csr &M, tsg_dev_tiles &t, uint16_t **mask_out, hipStream_t s);
// whether every CSR row is column-sorted (synchronous)
int dev_rows_sorted(Context &cx, const tsg_dev_csr &M, bool *sorted, hipStream_t s);
int dev_rows_sorted_async(Context &cx, const tsg_dev_csr &M, int *host_flag, hipStream_t s);
// the same check with its last step left to the caller: the per-workgroup shares
// (pool-owned part, nb of them) are summed either by dev_rows_sorted_finish or
// inside the row-merge setup's binning kernel (one launch fewer)
struct SortedShares {
    int *part = nullptr;
    int nb = 0;
    int *dflag = nullptr;  // device view of the host flag
};
int dev_rows_sorted_shares(Context &cx, const tsg_dev_csr &M, int *host_flag, SortedShares *sh, hipStream_t s);
int dev_rows_sorted_finish(Context &cx, SortedShares &sh, hipStream_t s);
// the same for the B rows A references only (row-merge / band paths)
int dev_rows_sorted_shares_ref(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, int *host_flag,
                               SortedShares *sh, hipStream_t s);
int dev_tile2csr(Context &cx, const tsg_dev_tiles &C, tsg_dev_csr &out, hipStream_t s);
// banded path (tsg_band.hip): every C row's reachable columns within one
// window of <= 2,048 columns, the windows holding at least as many products as
// columns in all (FEM-like operands; force: any density).  BandWin holds the
// check's results for the product (caller-owned device arrays: win, width).
struct BandWin {
    int2 *win = nullptr;         // per row: first and last reachable column
    long long *width = nullptr;  // per row: window width (+1 slot), scanned into staging offsets
    long long products = 0;      // element products (nnzCub)
    long long wcols = 0;         // window columns in all (bounds nnz(C))
    int2 *ebnd = nullptr;        // per A entry: its B row's [start, end) (the statistics kernel's by-product)
};
// sh (optional): B's sortedness shares, summed by the check's last kernel (and released)
int dev_band_check(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, bool force, bool *ok, BandWin *bw,
                   hipStream_t s, SortedShares *sh = nullptr);
int dev_spgemm_band(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, BandWin &bw, tsg_dev_csr &C,
                    tsg_stats *st, hipStream_t s, hipEvent_t *ev);
// row-merge path (tsg_rows.hip): CSR in -> CSR out, B's rows column-sorted;
// rows binned by element products, each row's B rows merged (or, for the
// longest rows, marked in an LDS column bitmap).  Two halves around the
// caller's one host round trip: the setup (entry table, classes, routing
// statistics), then the run.
struct RowsPlan {
    int2 *ebnd = nullptr;      // per A entry: its B row's [start, end)
    long long *E = nullptr;    // per A entry: prefix of the element products
    int4 *lists = nullptr;     // the classes' rows: (row, its first A entry, its A entries, -)
    long long *soff = nullptr; // per row: staging offset
    int *cls = nullptr;        // class counts + statistics (device)
    int *rowpointer = nullptr; // C's row pointers (row counts until the scan)
    int ncls[8] = {};
    long long products = 0, hprod = 0, pmax = 0;  // all / class-H rows' products, the longest row's
    long long hubprod = 0;     // hub rows' products (past kRowsHubProducts)
    long long hk = 0;          // class-H rows with more runs than the one-walk kernel takes
    long long hbig = 0;        // class-H rows' products past the one-walk register share (their scratch)
};
// Class-H rows past kRowsHubProducts products are hub rows: one run holding all
// but 4,096 of them -> the dominant-run kernels (k_rows_dr_*); the other hub
// rows and the rows past the one-walk kernel's runs or column span -> the
// windowed kernels (k_rows_w*: (row, column window) units); the rest the
// one-walk bitmap kernel (k_rows_bitmap).
constexpr long long kRowsHubProducts = 65536;
// the row-merge path sizes C by the products (no read-back of nnz(C) before the
// compaction) while their 12 B each stay within this; past it C is sized exactly
// (peak device memory of the path: 12 B per product of staging + C + the A
// entry table)
constexpr long long kRowsProductSizedC = 8LL << 30;
// sh (optional): B's sortedness shares, summed by the binning kernel (and released)
int dev_rows_setup_async(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, RowsPlan &p, hipStream_t s,
                         SortedShares *sh = nullptr);
void dev_rows_setup_read(Context &cx, RowsPlan &p);  // after the stream synchronised
bool dev_rows_accept(const RowsPlan &p);
void dev_rows_release(Context &cx, RowsPlan &p);
// ev (optional): 1 set up | 4..5 the row kernels | 3 end
int dev_rows_run(Context &cx, const tsg_dev_csr &A, const tsg_dev_csr &B, RowsPlan &p, tsg_dev_csr &C,
                 tsg_stats *st, hipStream_t s, hipEvent_t *ev);
// two-launch exclusive scans (tsg_rows.hip) for up to 2,048 tiles of 4,096
// values (TSG_ERR_UNSUPPORTED past it): i64 in place; row pointers (n = m + 1)
// with nnz(C) stored into the host-mapped *hnnz_dev by the kernel
int dev_scan_i64_fused(Context &cx, long long *a, long n, hipStream_t s);
int dev_scan_rows_fused(Context &cx, int *rp, int m, int *hnnz_dev, hipStream_t s);
// exclusive scan (n+1 idiom) whose total is read back
int scan_exclusive_i32_total(Context &cx, int *a, long n, hipStream_t s, long long *total);

// read a device int / long long synchronously through pinned memory
int read_i32(Context &cx, const int *d, int *h, hipStream_t s);
int read_i64(Context &cx, const long long *d, long long *h, hipStream_t s);

bool tile_size_supported(int tm, int tn);  // the SpGEMM steps (16x16)
bool tile_side_supported(int t);         // csr2tile / tile2csr sides: 16, 32, 48, 64

}  // namespace tsg
