/*
 * tsg.h -- C ABI of the MI355X-native TileSpGEMM (libtsg.so).
 *
 * Drop-in for the GPU path of for-the-juan/SpGEMM (a TileSpGEMM fork).  Plain C
 * types only: int / pointers / sizes, no torch or HIP types in the signatures
 * (a stream is passed as `void *` = hipStream_t).  Every function returns an int
 * status (TSG_OK = 0, negative on error) and never calls exit().
 *
 * Two layers:
 *  (1) Host-pointer functions with the reference's names and argument meaning
 *      (callee allocates outputs with malloc, caller owns them; free with
 *      tsg_matrix_destroy / tsg_csr_free).  Each runs the hand-written gfx950
 *      HIP kernels; host<->device copies happen inside, as in the reference.
 *  (2) Device-resident functions (tsg_dev_*) on a tsg_context: device pointers
 *      in and out, one explicit stream, outputs owned by the context.
 *
 * The library fails loudly (TSG_ERR_NO_DEVICE) when no HIP device is present:
 * there is no CPU fallback.
 */
#ifndef TSG_H
#define TSG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSG_OK 0
#define TSG_ERR_INVALID (-1)     /* bad argument / tile size / shape             */
#define TSG_ERR_HIP (-2)         /* a HIP runtime call failed                    */
#define TSG_ERR_OOM (-3)         /* device or host allocation failed             */
#define TSG_ERR_OVERFLOW (-4)    /* a count exceeds the int32 layout fields       */
#define TSG_ERR_NO_DEVICE (-5)   /* no HIP device visible                         */
#define TSG_ERR_UNSUPPORTED (-6) /* shape/tile size not built into this library   */
#define TSG_ERR_IO (-7)          /* Matrix-Market read failure                    */

/* Field-for-field the reference SMatrix (src/common.h:150-172), so a caller's
 * SMatrix* can be passed as tsg_smatrix* unchanged.  Tile index types are
 * uint16_t as in src/common.h:140-146. */
typedef struct tsg_smatrix {
    int m;
    int n;
    int nnz;
    int isSymmetric;
    double *value;
    int *columnindex;
    int *rowpointer;
    int tilem;
    int tilen;
    int *tile_ptr;
    int *tile_columnidx;
    int *tile_rowidx;
    int *tile_nnz;
    int numtile;
    double *tile_csr_Value;
    uint16_t *tile_csr_Col;
    uint16_t *tile_csr_Ptr;
    uint16_t *mask;
    int *csc_tile_ptr;
    int *csc_tile_rowidx;
} tsg_smatrix;

/* Per-call measurements (device timestamps from HIP events on the call's stream). */
typedef struct tsg_stats {
    double t_csr2tile_ms;  /* GPU csr2tile of A and B                          */
    double t_step1_ms;     /* tile-level symbolic (C tile structure)            */
    double t_step2_ms;     /* per-tile bitmask symbolic + nnz scan              */
    double t_step3_ms;     /* per-tile numeric                                  */
    double t_tile2csr_ms;  /* GPU tile2csr                                      */
    double t_malloc_ms;    /* host-side allocation + size read-back stalls      */
    double t_kern_ms;      /* steps 1-3 incl. allocation (reference's timer)     */
    double t_e2e_ms;       /* device CSR in -> device CSR out                   */
    long long nnzCub;      /* sum_{a in A} rowlen_B(col(a))                     */
    long long numtileA, numtileB, numblkC, nnzC;  /* numtileB = -1: not counted (B too wide
                                                      for the count units; CSR path only) */
    long long tile_products; /* tile-level intermediate products (step-1 work)  */
    double t_step3_kernel_ms;  /* the step-3 numeric kernel alone (dominant kernel) */
    long long path;            /* the CSR path that ran: TSG_PATH_TILES / _BAND / _ROWS */
} tsg_stats;

/* tsg_stats.path (the CSR-in -> CSR-out routing) */
#define TSG_PATH_TILES 0  /* staged tile pipeline: csr2tile structure, steps 1-3, tile2csr */
/* 1: retired (the fused element path of rounds 1-3; the row-merge path is faster on short rows too) */
#define TSG_PATH_BAND 2   /* banded rows: dense LDS window per row */
#define TSG_PATH_ROWS 3   /* row merge: rows binned by products, B runs merged in LDS */

/* ---------------- library / device ---------------- */
const char *tsg_version(void);
int tsg_device_count(int *count);
const char *tsg_status_string(int status);

/* ---------------- layer 1: reference-named host functions ---------------- */

/* Matrix-Market reader with mmio_allinone's exact CSR order
 * (src/mmio_highlevel.h:593-759): counting sort by row, in-row file order,
 * symmetric/hermitian mirrored in file order, pattern -> 1.0. */
int tsg_mmio_allinone(const char *filename, tsg_smatrix *A);

/* value[k] = k % 10 by CSR position (src/main.cu:111-112). */
void tsg_values_pos_mod10(tsg_smatrix *A);

/* Stable CSR->CSC transpose on the GPU (replaces matrix_transposition,
 * src/utils.h:161-198).  Writes B := A^T as a new malloc'd CSR. */
int tsg_transpose(const tsg_smatrix *A, tsg_smatrix *B);

/* sum_{a in A} rowlen_B(col(a)) on the GPU (src/main.cu:155-162). */
int tsg_nnzcub(const tsg_smatrix *A, const tsg_smatrix *B, unsigned long long *nnzCub);

/* Replaces csr2tile_row_major (src/csr2tile.h:205).  Fills the tile fields of A
 * (tile_ptr, tile_columnidx, tile_rowidx, tile_nnz, tile_csr_Ptr [numtile*tm],
 * tile_csr_Col = r*tn+c, tile_csr_Value, mask). */
int tsg_csr2tile_row_major(tsg_smatrix *A, int tile_size_m, int tile_size_n);

/* Replaces csr2tile_col_major (src/csr2tile.h:279).  B tiles are tn x tm:
 * row-major structure (tile_ptr/tile_columnidx), CSC structure
 * (csc_tile_ptr/csc_tile_rowidx), payload in CSC tile order (tile_nnz,
 * tile_csr_Ptr [numtile*tn], tile_csr_Col = local col, tile_csr_Value, mask). */
int tsg_csr2tile_col_major(tsg_smatrix *B, int tile_size_m, int tile_size_n);

/* Replaces tilespgemm (src/tilespgemm-cuda.h:2220-2235), same argument list.
 * blk_intersec_bitmask_A/B may be NULL (they are not needed by this
 * implementation; the reference builds them on the host, src/main.cu:194-232).
 * Fills C's tile fields (tile_ptr, tile_columnidx, tile_rowidx, tile_nnz
 * exclusive [numblkC+1], tile_csr_Ptr [numblkC*tm], tile_csr_Col,
 * tile_csr_Value, mask) plus m, n, tilem, tilen, numtile, nnz.  Structurally
 * empty C tiles (step-1 tiles whose element product is empty) are kept with
 * nnz 0 and an all-zero Ptr, exactly the reference's C tile list.
 * filename is only echoed in the printed lines (may be NULL). */
int tsg_tilespgemm(tsg_smatrix *A, tsg_smatrix *B, tsg_smatrix *C,
                   unsigned int *blk_intersec_bitmask_A, unsigned int *blk_intersec_bitmask_B,
                   int blk_intersec_bitmask_len, double densityA, double densityB,
                   unsigned long long nnzCub, unsigned long long *nnzC_computed,
                   double *compression_rate, double *time_tile, double *gflops_tile,
                   const char *filename, double *time_step1, double *time_step2,
                   double *time_step3, double *time_malloc, int tile_size_m, int tile_size_n);

/* Replaces tile2csr (src/tile2csr.h:72-140), called as tile2csr(C, tm, tm). */
int tsg_tile2csr(tsg_smatrix *C, int tile_size_m, int tile_size_n);

/* One shot CSR -> CSR: C = A * B, fp64, structural pattern (no zero dropping),
 * ascending columns.  Uploads A and B and runs tsg_dev_spgemm (below) -- the
 * routed device pipeline (row-merge, banded or staged tile path, whichever
 * its statistics pick; stats->path says which) -- then downloads C.  The same C
 * as csr2tile + steps 1-3 + tile2csr.  C->rowpointer/columnindex/value are
 * malloc'd. stats may be NULL. */
int tsg_spgemm_csr(const tsg_smatrix *A, const tsg_smatrix *B, tsg_smatrix *C,
                   int tile_size_m, int tile_size_n, tsg_stats *stats);

/* Frees every non-NULL pointer field and zeroes the struct (covers the
 * reference's matrix_destroy, src/csr2tile.h:509-518, and the CSR arrays). */
void tsg_matrix_destroy(tsg_smatrix *M);

/* ---------------- layer 2: device-resident API ---------------- */
typedef struct tsg_context tsg_context;

/* Device CSR: pointers are device memory. */
typedef struct tsg_dev_csr {
    int m, n, nnz;
    int *rowpointer;
    int *columnindex;
    double *value;
} tsg_dev_csr;

/* Device tiled matrix (the reference's tile fields, device memory).  For a
 * col-major (B) tiling, csc_* and tile_rm2csc are set. */
typedef struct tsg_dev_tiles {
    int m, n, nnz;
    int tile_m, tile_n;        /* rows / cols of one tile                     */
    int tilem, tilen, numtile;
    int *tile_ptr;
    int *tile_columnidx;
    int *tile_rowidx;
    int *tile_nnz;
    uint16_t *tile_csr_Ptr;
    uint16_t *tile_csr_Col;
    double *tile_csr_Value;
    uint16_t *mask;
    int *csc_tile_ptr;
    int *csc_tile_rowidx;
    int *tile_rm2csc;          /* row-major tile index -> CSC tile index      */
    uint16_t *rm_mask;         /* B only: tile masks in row-major tile order   */
    int *rm_rowstart;          /* B only: per row-major tile, tile_n+1 absolute
                                  row starts into the CSC-ordered payload      */
} tsg_dev_tiles;

/* A context owns a device, a caching device allocator and the outputs of the
 * tsg_dev_* calls made on it.  One stream per call; not thread-safe per context. */
int tsg_context_create(int device, tsg_context **ctx);
int tsg_context_destroy(tsg_context *ctx);
/* Returns every context-owned output/temporary block to the cache. */
int tsg_context_reset(tsg_context *ctx);

int tsg_dev_csr2tile_row_major(tsg_context *ctx, const tsg_dev_csr *A, int tile_size_m,
                               int tile_size_n, void *stream, tsg_dev_tiles *out);
int tsg_dev_csr2tile_col_major(tsg_context *ctx, const tsg_dev_csr *B, int tile_size_m,
                               int tile_size_n, void *stream, tsg_dev_tiles *out);
int tsg_dev_tilespgemm(tsg_context *ctx, const tsg_dev_tiles *A, const tsg_dev_tiles *B,
                       void *stream, tsg_dev_tiles *C, tsg_stats *stats);
int tsg_dev_tile2csr(tsg_context *ctx, const tsg_dev_tiles *C, void *stream, tsg_dev_csr *out);
int tsg_dev_transpose(tsg_context *ctx, const tsg_dev_csr *A, void *stream, tsg_dev_csr *out);
/* Full pipeline, device CSR in -> device CSR out (outputs owned by ctx). */
int tsg_dev_spgemm(tsg_context *ctx, const tsg_dev_csr *A, const tsg_dev_csr *B,
                   int tile_size_m, int tile_size_n, void *stream, tsg_dev_csr *C,
                   tsg_stats *stats);
/* Whether every row of M is strictly column-sorted (*sorted = 1, else 0): the
 * check tsg_dev_spgemm makes on B on every call (the row-merge and banded
 * routes need it), on its own. */
int tsg_dev_csr_rows_sorted(tsg_context *ctx, const tsg_dev_csr *M, void *stream, int *sorted);
/* tsg_dev_spgemm for a B whose rows the caller has found column-sorted
 * (tsg_dev_csr_rows_sorted returned 1 and B has not changed since; the
 * caller's contract -- an unsorted B passed here gives a wrong C): the
 * per-call check of B is skipped, so a sequence of row blocks of A against one
 * B checks B once.  b_checked_sorted = 0 is tsg_dev_spgemm itself. */
int tsg_dev_spgemm_sorted_b(tsg_context *ctx, const tsg_dev_csr *A, const tsg_dev_csr *B,
                            int b_checked_sorted, int tile_size_m, int tile_size_n, void *stream,
                            tsg_dev_csr *C, tsg_stats *stats);
/* Copies between host and device (stream-ordered, synchronous on return). */
int tsg_memcpy_h2d(tsg_context *ctx, void *dst, const void *src, size_t bytes, void *stream);
int tsg_memcpy_d2h(tsg_context *ctx, void *dst, const void *src, size_t bytes, void *stream);
int tsg_memcpy_d2d(tsg_context *ctx, void *dst, const void *src, size_t bytes, void *stream);
int tsg_dev_malloc(tsg_context *ctx, void **ptr, size_t bytes);
int tsg_dev_free(tsg_context *ctx, void *ptr);

#ifdef __cplusplus
}
#endif
#endif /* TSG_H */
