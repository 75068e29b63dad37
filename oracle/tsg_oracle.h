/*
 * tsg_oracle.h -- CPU ORACLE for the TileSpGEMM hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a clean-room C restatement of the reference's host algorithms
 * (for-the-juan/SpGEMM, read-only at /root/reference).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / reported CPU baseline -- never as the thing measured or
 * shipped.  The product (libtsg.so) does not link it.
 *
 * Parity pins: the restatement is checked against the reference's own host code
 * compiled in this container (oracle/_ref, see oracle/Makefile) on the
 * UnitTest/CSR2TILE fixtures; the outputs are frozen as tests/golden/*.npz.
 */
#ifndef TSG_ORACLE_H
#define TSG_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Field-for-field the reference SMatrix (src/common.h:150-172). */
typedef struct {
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
} tsgo_mat;

/* mmio_allinone (src/mmio_highlevel.h:593-759): CSR with file-order rows. 0 = ok. */
int tsgo_mmio_load(const char *path, tsgo_mat *A);
/* value[k] = k % 10 by CSR position (src/main.cu:111-112). */
void tsgo_values_pos_mod10(tsgo_mat *A);
/* Stable counting transpose (src/utils.h:161-198). Output arrays caller-sized. */
void tsgo_transpose(int m, int n, int nnz, const int *rowptr, const int *col,
                    const double *val, int *cscColPtr, int *cscRowIdx, double *cscVal);
/* B := A^T as a new CSR (src/main.cu:126-139). */
int tsgo_make_transpose(const tsgo_mat *A, tsgo_mat *B);
/* sum_{a in A} rowlen_B(col(a))  (src/main.cu:155-162). */
unsigned long long tsgo_nnzcub(const tsgo_mat *A, const tsgo_mat *B);

/* csr2tile_row_major (src/csr2tile.h:205-277). */
int tsgo_csr2tile_row_major(tsgo_mat *A, int tm, int tn);
/* csr2tile_col_major (src/csr2tile.h:279-506). */
int tsgo_csr2tile_col_major(tsgo_mat *B, int tm, int tn);

/* Tiled C = A * B with the reference's output layout (src/tilespgemm-cuda.h:2220-2844):
 * tile_ptr/tile_columnidx/tile_rowidx/tile_nnz(exclusive)/tile_csr_Ptr/Col/Value/mask.
 * Values are the mathematically correct sums. */
int tsgo_tilespgemm(const tsgo_mat *A, const tsgo_mat *B, tsgo_mat *C, int tm, int tn);
/* tile2csr (src/tile2csr.h:72-140): fills C->rowpointer/columnindex/value/nnz. */
int tsgo_tile2csr(tsgo_mat *C, int tm, int tn);

/* spgemm_spa (src/spgemm_serialref_spa_new.h:7-105), OpenMP, symbolic only.
 * rowptrC has mA+1 entries.  If get_nnzC_only, fills rowptrC (exclusive) and *nnzC.
 * Otherwise fills colidxC (ascending per row) using rowptrC from the first call.
 * row_begin/row_end restrict the rows processed (bounded CPU-baseline samples);
 * pass 0, mA for all rows.  Returns -2 when nnz(C) of the rows exceeds int32. */
int tsgo_spa(const tsgo_mat *A, const tsgo_mat *B, int *rowptrC, int *colidxC,
             long long *nnzC, int get_nnzC_only, int row_begin, int row_end);

/* Numeric Gustavson with a dense row accumulator
 * (src/external/cusparse/spgemm_serialref_spa.h:7-119), OpenMP.
 * Structural pattern (no zero dropping), ascending columns.  Allocates C CSR. */
int tsgo_gustavson(const tsgo_mat *A, const tsgo_mat *B, tsgo_mat *C);
/* Same restricted to rows [row_begin,row_end): returns nnz of those rows only
 * (used for bounded timing samples; C arrays not kept). */
long long tsgo_gustavson_rows(const tsgo_mat *A, const tsgo_mat *B, int row_begin, int row_end);

void tsgo_free(tsgo_mat *M);
int tsgo_num_threads(void);

#ifdef __cplusplus
}
#endif
#endif
