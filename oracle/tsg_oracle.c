/*
 * tsg_oracle.c -- CPU ORACLE for the TileSpGEMM hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room restatement of the reference's host algorithms.  Every function
 * cites the reference file:line it follows (paths under /root/reference/).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this
 * library; the product (spgemm_amd/lib/libtsg.so) never does.
 *
 * Parity pins: checked against oracle/_ref (the reference's own host code,
 * compiled here by oracle/Makefile) on the reference's UnitTest/CSR2TILE
 * fixtures; frozen outputs live in tests/golden/.
 */
#include "tsg_oracle.h"

#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MASK_BITS 16

static void *xcalloc(size_t n, size_t sz) {
    if (n == 0) n = 1;
    return calloc(n, sz);
}

int tsgo_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* in-place exclusive scan over `len` ints (src/utils.h:36-51) */
static void excl_scan_int(int *a, long len) {
    int run = 0;
    for (long i = 0; i < len; i++) {
        int v = a[i];
        a[i] = run;
        run += v;
    }
}

/* ------------------------------------------------------------------------ */
/* Matrix-Market load: src/mmio_highlevel.h:593-759 (+ banner src/mmio.h:398,
 * size line src/mmio.h:568).  Rows by counting sort, in-row order = file order;
 * symmetric/hermitian: each off-diagonal (i,j) also emits (j,i), both placed in
 * file order (mmio_highlevel.h:707-731); pattern -> 1.0. */
int tsgo_mmio_load(const char *path, tsgo_mat *A) {
    memset(A, 0, sizeof(*A));
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char line[1025], t0[64], t1[64], t2[64], t3[64], t4[64];
    if (!fgets(line, sizeof line, f)) { fclose(f); return -2; }
    if (sscanf(line, "%63s %63s %63s %63s %63s", t0, t1, t2, t3, t4) != 5) { fclose(f); return -2; }
    for (char *p = t1; *p; p++) *p = (char)tolower(*p);
    for (char *p = t2; *p; p++) *p = (char)tolower(*p);
    for (char *p = t3; *p; p++) *p = (char)tolower(*p);
    for (char *p = t4; *p; p++) *p = (char)tolower(*p);
    if (strncmp(t0, "%%MatrixMarket", 14) != 0 || strcmp(t1, "matrix") != 0) { fclose(f); return -2; }
    if (strcmp(t2, "coordinate") != 0) { fclose(f); return -3; }
    int is_real = !strcmp(t3, "real"), is_cplx = !strcmp(t3, "complex");
    int is_int = !strcmp(t3, "integer"), is_pat = !strcmp(t3, "pattern");
    if (!(is_real || is_cplx || is_int || is_pat)) { fclose(f); return -3; }
    int sym = !strcmp(t4, "symmetric") || !strcmp(t4, "hermitian");
    int m = 0, n = 0, nz = 0;
    do {
        if (!fgets(line, sizeof line, f)) { fclose(f); return -4; }
    } while (line[0] == '%');
    if (sscanf(line, "%d %d %d", &m, &n, &nz) != 3) { fclose(f); return -4; }

    int *ri = (int *)xcalloc(nz, sizeof(int)), *ci = (int *)xcalloc(nz, sizeof(int));
    double *vv = (double *)xcalloc(nz, sizeof(double));
    int *cnt = (int *)xcalloc((size_t)m + 1, sizeof(int));
    for (int k = 0; k < nz; k++) {
        int i = 0, j = 0, iv = 0;
        double x = 1.0, xi = 0.0;
        int got;
        if (is_real) got = fscanf(f, "%d %d %lg", &i, &j, &x);
        else if (is_cplx) got = fscanf(f, "%d %d %lg %lg", &i, &j, &x, &xi);
        else if (is_int) { got = fscanf(f, "%d %d %d", &i, &j, &iv); x = iv; }
        else { got = fscanf(f, "%d %d", &i, &j); x = 1.0; }
        if (got < 2 || i < 1 || j < 1 || i > m || j > n) {
            free(ri); free(ci); free(vv); free(cnt); fclose(f); return -5;
        }
        ri[k] = i - 1;
        ci[k] = j - 1;
        vv[k] = x;
        cnt[i - 1]++;
    }
    fclose(f);
    if (sym)
        for (int k = 0; k < nz; k++)
            if (ri[k] != ci[k]) cnt[ci[k]]++;
    excl_scan_int(cnt, (long)m + 1);
    int total = cnt[m];
    int *rowptr = (int *)xcalloc((size_t)m + 1, sizeof(int));
    memcpy(rowptr, cnt, ((size_t)m + 1) * sizeof(int));
    int *fill = (int *)xcalloc((size_t)m + 1, sizeof(int));
    int *col = (int *)xcalloc(total, sizeof(int));
    double *val = (double *)xcalloc(total, sizeof(double));
    for (int k = 0; k < nz; k++) {
        int p = rowptr[ri[k]] + fill[ri[k]]++;
        col[p] = ci[k];
        val[p] = vv[k];
        if (sym && ri[k] != ci[k]) {
            p = rowptr[ci[k]] + fill[ci[k]]++;
            col[p] = ri[k];
            val[p] = vv[k];
        }
    }
    free(ri); free(ci); free(vv); free(cnt); free(fill);
    A->m = m; A->n = n; A->nnz = total; A->isSymmetric = sym;
    A->rowpointer = rowptr; A->columnindex = col; A->value = val;
    return 0;
}

/* src/main.cu:111-112 */
void tsgo_values_pos_mod10(tsgo_mat *A) {
    for (int k = 0; k < A->nnz; k++) A->value[k] = (double)(k % 10);
}

/* src/utils.h:161-198: histogram of columns, exclusive scan, row-ordered insert. */
void tsgo_transpose(int m, int n, int nnz, const int *rowptr, const int *col,
                    const double *val, int *cscColPtr, int *cscRowIdx, double *cscVal) {
    (void)nnz;
    memset(cscColPtr, 0, ((size_t)n + 1) * sizeof(int));
    for (int r = 0; r < m; r++)
        for (int p = rowptr[r]; p < rowptr[r + 1]; p++) cscColPtr[col[p]]++;
    excl_scan_int(cscColPtr, (long)n + 1);
    int *next = (int *)xcalloc((size_t)n + 1, sizeof(int));
    memcpy(next, cscColPtr, ((size_t)n + 1) * sizeof(int));
    for (int r = 0; r < m; r++)
        for (int p = rowptr[r]; p < rowptr[r + 1]; p++) {
            int q = next[col[p]]++;
            cscRowIdx[q] = r;
            if (val) cscVal[q] = val[p];
        }
    free(next);
}

/* src/main.cu:126-139 */
int tsgo_make_transpose(const tsgo_mat *A, tsgo_mat *B) {
    memset(B, 0, sizeof(*B));
    B->m = A->n; B->n = A->m; B->nnz = A->nnz;
    B->rowpointer = (int *)xcalloc((size_t)A->n + 1, sizeof(int));
    B->columnindex = (int *)xcalloc(A->nnz, sizeof(int));
    B->value = (double *)xcalloc(A->nnz, sizeof(double));
    tsgo_transpose(A->m, A->n, A->nnz, A->rowpointer, A->columnindex, A->value,
                   B->rowpointer, B->columnindex, B->value);
    return 0;
}

/* src/main.cu:155-162 */
unsigned long long tsgo_nnzcub(const tsgo_mat *A, const tsgo_mat *B) {
    unsigned long long s = 0;
    for (int p = 0; p < A->nnz; p++) {
        int k = A->columnindex[p];
        s += (unsigned long long)(B->rowpointer[k + 1] - B->rowpointer[k]);
    }
    return s;
}

/* ------------------------------------------------------------------------ */
/* Shared helper: the tile structure of a CSR cut into (rows_per_tile x
 * cols_per_tile) tiles -- tile_ptr (exclusive), tile_columnidx ascending per
 * tile row, tile_rowidx.  Mirrors step1_kernel/step2_kernel's structure output
 * (src/csr2tile.h:6-110) and the per-row sort (:235-239). */
static int tile_structure(int m, int n, const int *rowptr, const int *col, int rpt, int cpt,
                          int *tilem_out, int *tilen_out, int **tile_ptr_out,
                          int **tile_col_out, int **tile_row_out) {
    int tilem = (m + rpt - 1) / rpt, tilen = (n + cpt - 1) / cpt;
    int *tile_ptr = (int *)xcalloc((size_t)tilem + 1, sizeof(int));
#pragma omp parallel
    {
        unsigned char *seen = (unsigned char *)xcalloc((size_t)tilen, 1);
#pragma omp for schedule(dynamic, 256)
        for (int ti = 0; ti < tilem; ti++) {
            int r0 = ti * rpt, r1 = (ti + 1) * rpt < m ? (ti + 1) * rpt : m;
            for (int p = rowptr[r0]; p < rowptr[r1]; p++) {
                int tc = col[p] / cpt;
                if (!seen[tc]) { seen[tc] = 1; tile_ptr[ti]++; }
            }
            for (int p = rowptr[r0]; p < rowptr[r1]; p++) seen[col[p] / cpt] = 0;
        }
        free(seen);
    }
    excl_scan_int(tile_ptr, (long)tilem + 1);
    int numtile = tile_ptr[tilem];
    int *tcol = (int *)xcalloc(numtile, sizeof(int));
    int *trow = (int *)xcalloc(numtile, sizeof(int));
#pragma omp parallel
    {
        unsigned char *seen = (unsigned char *)xcalloc((size_t)tilen, 1);
#pragma omp for schedule(dynamic, 256)
        for (int ti = 0; ti < tilem; ti++) {
            int r0 = ti * rpt, r1 = (ti + 1) * rpt < m ? (ti + 1) * rpt : m;
            for (int p = rowptr[r0]; p < rowptr[r1]; p++) seen[col[p] / cpt] = 1;
            /* ascending tile columns == the blkj loop of step2_kernel (:92-105) */
            int w = tile_ptr[ti];
            for (int p = rowptr[r0]; p < rowptr[r1]; p++) {
                int tc = col[p] / cpt;
                if (seen[tc] == 1) { seen[tc] = 2; tcol[w++] = tc; }
            }
            /* insertion sort of this tile row's columns (small) */
            for (int a = tile_ptr[ti] + 1; a < w; a++) {
                int x = tcol[a], b = a - 1;
                while (b >= tile_ptr[ti] && tcol[b] > x) { tcol[b + 1] = tcol[b]; b--; }
                tcol[b + 1] = x;
            }
            for (int a = tile_ptr[ti]; a < w; a++) { trow[a] = ti; seen[tcol[a]] = 0; }
        }
        free(seen);
    }
    *tilem_out = tilem; *tilen_out = tilen;
    *tile_ptr_out = tile_ptr; *tile_col_out = tcol; *tile_row_out = trow;
    return numtile;
}

static int find_tile(const int *cols, int lo, int hi, int key) {
    while (lo < hi) {
        int mid = lo + (hi - lo) / 2;
        if (cols[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* csr2tile_row_major: src/csr2tile.h:205-277 (step kernels :6-203).
 * Payload order inside a tile: row-major, CSR order inside a row (:152-168);
 * tile_csr_Col = r*tn + c (:192); mask bit 15 - c%16, MSB first (:193-195). */
int tsgo_csr2tile_row_major(tsgo_mat *A, int tm, int tn) {
    if (tm <= 0 || tn <= 0 || tm % MASK_BITS || tn % MASK_BITS) return -1;
    A->numtile = tile_structure(A->m, A->n, A->rowpointer, A->columnindex, tm, tn,
                                &A->tilem, &A->tilen, &A->tile_ptr, &A->tile_columnidx,
                                &A->tile_rowidx);
    int numtile = A->numtile, wpr = tn / MASK_BITS;
    A->tile_nnz = (int *)xcalloc((size_t)numtile + 1, sizeof(int));
    A->tile_csr_Ptr = (uint16_t *)xcalloc((size_t)numtile * tm, sizeof(uint16_t));
    A->tile_csr_Col = (uint16_t *)xcalloc(A->nnz, sizeof(uint16_t));
    A->tile_csr_Value = (double *)xcalloc(A->nnz, sizeof(double));
    A->mask = (uint16_t *)xcalloc((size_t)numtile * tm * wpr, sizeof(uint16_t));
    /* pass 1: per (tile,row) counts */
    for (int ti = 0; ti < A->tilem; ti++) {
        int t0 = A->tile_ptr[ti], t1 = A->tile_ptr[ti + 1];
        for (int r = 0; r < tm && ti * tm + r < A->m; r++) {
            int R = ti * tm + r;
            for (int p = A->rowpointer[R]; p < A->rowpointer[R + 1]; p++) {
                int t = find_tile(A->tile_columnidx, t0, t1, A->columnindex[p] / tn);
                A->tile_nnz[t]++;
                A->tile_csr_Ptr[(size_t)t * tm + r]++;
            }
        }
    }
    excl_scan_int(A->tile_nnz, (long)numtile + 1);
    for (int t = 0; t < numtile; t++) {
        int run = 0;
        for (int r = 0; r < tm; r++) {
            int v = A->tile_csr_Ptr[(size_t)t * tm + r];
            A->tile_csr_Ptr[(size_t)t * tm + r] = (uint16_t)run;
            run += v;
        }
    }
    /* pass 2: place in traversal order with a running counter per tile */
    int *fill = (int *)xcalloc(numtile, sizeof(int));
    for (int ti = 0; ti < A->tilem; ti++) {
        int t0 = A->tile_ptr[ti], t1 = A->tile_ptr[ti + 1];
        for (int r = 0; r < tm && ti * tm + r < A->m; r++) {
            int R = ti * tm + r;
            for (int p = A->rowpointer[R]; p < A->rowpointer[R + 1]; p++) {
                int c = A->columnindex[p];
                int t = find_tile(A->tile_columnidx, t0, t1, c / tn);
                int lc = c - (c / tn) * tn;
                int q = A->tile_nnz[t] + fill[t]++;
                A->tile_csr_Col[q] = (uint16_t)(r * tn + lc);
                A->tile_csr_Value[q] = A->value[p];
                A->mask[(size_t)t * tm * wpr + (size_t)r * wpr + lc / MASK_BITS] |=
                    (uint16_t)(1u << (MASK_BITS - 1 - lc % MASK_BITS));
            }
        }
    }
    free(fill);
    return 0;
}

/* csr2tile_col_major: src/csr2tile.h:279-506.  B tiles are tn rows x tm cols.
 * Row-major tile structure (:328-388) for step 1; CSC tile structure = the
 * tiling of B^T (:287-347); payload in CSC tile order, each tile a CSR of its
 * tn local rows with ascending local col (per-tile transposes :390-484);
 * tile_csr_Col = plain local col; Ptr padded to tn rows (:480-483). */
int tsgo_csr2tile_col_major(tsgo_mat *B, int tm, int tn) {
    if (tm <= 0 || tn <= 0 || tm % MASK_BITS || tn % MASK_BITS) return -1;
    int m = B->m, n = B->n, wpr = tm / MASK_BITS;
    B->numtile = tile_structure(m, n, B->rowpointer, B->columnindex, tn, tm, &B->tilem,
                                &B->tilen, &B->tile_ptr, &B->tile_columnidx, &B->tile_rowidx);
    /* CSC of B (stable), then the tile structure of B^T */
    int *cptr = (int *)xcalloc((size_t)n + 1, sizeof(int));
    int *crow = (int *)xcalloc(B->nnz, sizeof(int));
    double *cval = (double *)xcalloc(B->nnz, sizeof(double));
    int *cpos = (int *)xcalloc(B->nnz, sizeof(int));
    tsgo_transpose(m, n, B->nnz, B->rowpointer, B->columnindex, B->value, cptr, crow, cval);
    {
        /* CSR position of each CSC entry (same stable order) */
        int *next = (int *)xcalloc((size_t)n + 1, sizeof(int));
        memcpy(next, cptr, ((size_t)n + 1) * sizeof(int));
        for (int r = 0; r < m; r++)
            for (int p = B->rowpointer[r]; p < B->rowpointer[r + 1]; p++) cpos[next[B->columnindex[p]]++] = p;
        free(next);
    }
    int bt_tilem, bt_tilen, *bt_row_unused;
    int nt2 = tile_structure(n, m, cptr, crow, tm, tn, &bt_tilem, &bt_tilen, &B->csc_tile_ptr,
                             &B->csc_tile_rowidx, &bt_row_unused);
    free(bt_row_unused);
    if (nt2 != B->numtile) return -2;
    int numtile = B->numtile;
    B->tile_nnz = (int *)xcalloc((size_t)numtile + 1, sizeof(int));
    B->tile_csr_Ptr = (uint16_t *)xcalloc((size_t)numtile * tn, sizeof(uint16_t));
    B->tile_csr_Col = (uint16_t *)xcalloc(B->nnz, sizeof(uint16_t));
    B->tile_csr_Value = (double *)xcalloc(B->nnz, sizeof(double));
    B->mask = (uint16_t *)xcalloc((size_t)numtile * tn * wpr, sizeof(uint16_t));
    /* counts per (csc tile, local row); tile columns own disjoint tiles */
#pragma omp parallel for schedule(dynamic, 64)
    for (int tj = 0; tj < B->tilen; tj++) {
        int t0 = B->csc_tile_ptr[tj], t1 = B->csc_tile_ptr[tj + 1];
        for (int c = tj * tm; c < (tj + 1) * tm && c < n; c++)
            for (int q = cptr[c]; q < cptr[c + 1]; q++) {
                int t = find_tile(B->csc_tile_rowidx, t0, t1, crow[q] / tn);
                B->tile_nnz[t]++;
                B->tile_csr_Ptr[(size_t)t * tn + crow[q] % tn]++;
            }
    }
    excl_scan_int(B->tile_nnz, (long)numtile + 1);
    for (int t = 0; t < numtile; t++) {
        int run = 0;
        for (int r = 0; r < tn; r++) {
            int v = B->tile_csr_Ptr[(size_t)t * tn + r];
            B->tile_csr_Ptr[(size_t)t * tn + r] = (uint16_t)run;
            run += v;
        }
    }
    /* fill: for each tile, rows ascending, local cols ascending, then CSR position:
     * iterate local cols ascending and rows ascending inside each column, and
     * insert into the (row) slot -- the per-tile transpose of :455-458 */
    int *rowfill = (int *)xcalloc((size_t)numtile * tn, sizeof(int));
#pragma omp parallel for schedule(dynamic, 64)
    for (int tj = 0; tj < B->tilen; tj++) {
        int t0 = B->csc_tile_ptr[tj], t1 = B->csc_tile_ptr[tj + 1];
        for (int c = tj * tm; c < (tj + 1) * tm && c < n; c++)
            for (int q = cptr[c]; q < cptr[c + 1]; q++) {
                int t = find_tile(B->csc_tile_rowidx, t0, t1, crow[q] / tn);
                int lr = crow[q] % tn, lc = c - tj * tm;
                int dst = B->tile_nnz[t] + B->tile_csr_Ptr[(size_t)t * tn + lr] +
                          rowfill[(size_t)t * tn + lr]++;
                B->tile_csr_Col[dst] = (uint16_t)lc;
                B->tile_csr_Value[dst] = cval[q];
                B->mask[(size_t)t * tn * wpr + (size_t)lr * wpr + lc / MASK_BITS] |=
                    (uint16_t)(1u << (MASK_BITS - 1 - lc % MASK_BITS));
            }
    }
    free(rowfill); free(cptr); free(crow); free(cval); free(cpos);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Tiled C = A*B.  Step 1 = tile-pattern product with a per-row SPA
 * (src/tilespgemm-cuda.h:279-392; the nsparse hash path gives the same sorted
 * list).  Step 2 = per C tile, k over A tile row i intersected with B tile
 * column j (CSC), maskC[r] |= maskB[c] for each A nonzero (r,c)
 * (:394-773); Ptr = exclusive scan of row popcounts, nnz = popcount
 * (:666-709).  Step 3 = values sum_k A(r,c)*B(c,x) at the mask positions,
 * local cols ascending per row (:1612-1952, correct arithmetic).  Tiles of the
 * structure whose product is empty keep nnz 0 and an all-zero Ptr.
 *
 * Evaluation order (OpenMP over C tile rows, so that full-size stand-ins run
 * in seconds): the matched (A tile, B tile) pairs of a tile row are visited
 * A tile by A tile (k ascending), each B tile of B's tile row k mapped to its
 * C tile -- for any one C tile the pairs still come k ascending, then the A
 * nonzeros in payload order, then the B row's entries, the order of the
 * per-tile accumulation above, so every value is the same sum. */
static int cmp_int_asc(const void *a, const void *b) {
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

int tsgo_tilespgemm(const tsgo_mat *A, const tsgo_mat *B, tsgo_mat *C, int tm, int tn) {
    memset(C, 0, sizeof(*C));
    if (A->n != B->m) return -1;
    int wpr = tm / MASK_BITS;
    int blkmA = A->tilem, blknB = B->tilen;
    C->m = A->m; C->n = B->n; C->tilem = blkmA; C->tilen = blknB;
    /* step 1: C tiles per tile row, then each row's columns ascending */
    C->tile_ptr = (int *)xcalloc((size_t)blkmA + 1, sizeof(int));
#pragma omp parallel
    {
        unsigned char *flag = (unsigned char *)xcalloc((size_t)blknB, 1);
#pragma omp for schedule(dynamic, 2)
        for (int i = 0; i < blkmA; i++) {
            int cnt = 0;
            for (int a = A->tile_ptr[i]; a < A->tile_ptr[i + 1]; a++) {
                int k = A->tile_columnidx[a];
                for (int b = B->tile_ptr[k]; b < B->tile_ptr[k + 1]; b++)
                    if (!flag[B->tile_columnidx[b]]) { flag[B->tile_columnidx[b]] = 1; cnt++; }
            }
            for (int a = A->tile_ptr[i]; a < A->tile_ptr[i + 1]; a++) {
                int k = A->tile_columnidx[a];
                for (int b = B->tile_ptr[k]; b < B->tile_ptr[k + 1]; b++) flag[B->tile_columnidx[b]] = 0;
            }
            C->tile_ptr[i] = cnt;
        }
        free(flag);
    }
    long total = 0;
    for (int i = 0; i < blkmA; i++) total += C->tile_ptr[i];
    if (total > 0x7fffffffL) return -3;
    excl_scan_int(C->tile_ptr, (long)blkmA + 1);
    int numblkC = C->tile_ptr[blkmA];
    C->numtile = numblkC;
    C->tile_columnidx = (int *)xcalloc(numblkC, sizeof(int));
    C->tile_rowidx = (int *)xcalloc(numblkC, sizeof(int));
#pragma omp parallel
    {
        unsigned char *flag = (unsigned char *)xcalloc((size_t)blknB, 1);
#pragma omp for schedule(dynamic, 2)
        for (int i = 0; i < blkmA; i++) {
            int w = C->tile_ptr[i];
            for (int a = A->tile_ptr[i]; a < A->tile_ptr[i + 1]; a++) {
                int k = A->tile_columnidx[a];
                for (int b = B->tile_ptr[k]; b < B->tile_ptr[k + 1]; b++) {
                    int j = B->tile_columnidx[b];
                    if (!flag[j]) { flag[j] = 1; C->tile_columnidx[w++] = j; }
                }
            }
            int t0 = C->tile_ptr[i];
            qsort(C->tile_columnidx + t0, (size_t)(w - t0), sizeof(int), cmp_int_asc);
            for (int t = t0; t < w; t++) { C->tile_rowidx[t] = i; flag[C->tile_columnidx[t]] = 0; }
        }
        free(flag);
    }

    /* step 2: masks (maskC[r] |= maskB[c] per matched pair and A nonzero), Ptr, nnz */
    C->tile_nnz = (int *)xcalloc((size_t)numblkC + 1, sizeof(int));
    C->tile_csr_Ptr = (uint16_t *)xcalloc((size_t)numblkC * tm, sizeof(uint16_t));
    C->mask = (uint16_t *)xcalloc((size_t)numblkC * tm * wpr, sizeof(uint16_t));
#pragma omp parallel
    {
        int *map = (int *)malloc(((size_t)blknB + 1) * sizeof(int));
        for (int j = 0; j < blknB; j++) map[j] = -1;
#pragma omp for schedule(dynamic, 2)
        for (int i = 0; i < blkmA; i++) {
            for (int t = C->tile_ptr[i]; t < C->tile_ptr[i + 1]; t++) map[C->tile_columnidx[t]] = t;
            for (int a = A->tile_ptr[i]; a < A->tile_ptr[i + 1]; a++) {
                int k = A->tile_columnidx[a];
                for (int brm = B->tile_ptr[k]; brm < B->tile_ptr[k + 1]; brm++) {
                    int j = B->tile_columnidx[brm], t = map[j];
                    int b0 = B->csc_tile_ptr[j], b1 = B->csc_tile_ptr[j + 1];
                    int b = find_tile(B->csc_tile_rowidx, b0, b1, k);  /* CSC payload id of tile (k, j) */
                    uint16_t *mc = C->mask + (size_t)t * tm * wpr;
                    const uint16_t *mb = B->mask + (size_t)b * tn * wpr;
                    for (int q = A->tile_nnz[a]; q < A->tile_nnz[a + 1]; q++) {
                        int r = A->tile_csr_Col[q] / tn, c = A->tile_csr_Col[q] % tn;
                        for (int w = 0; w < wpr; w++) mc[r * wpr + w] |= mb[c * wpr + w];
                    }
                }
            }
            for (int t = C->tile_ptr[i]; t < C->tile_ptr[i + 1]; t++) {
                const uint16_t *mc = C->mask + (size_t)t * tm * wpr;
                int nz = 0;
                for (int r = 0; r < tm; r++)
                    for (int w = 0; w < wpr; w++) nz += __builtin_popcount(mc[r * wpr + w]);
                if (nz) {
                    int run = 0;
                    for (int r = 0; r < tm; r++) {
                        C->tile_csr_Ptr[(size_t)t * tm + r] = (uint16_t)run;
                        for (int w = 0; w < wpr; w++) run += __builtin_popcount(mc[r * wpr + w]);
                    }
                }
                C->tile_nnz[t] = nz;
                map[C->tile_columnidx[t]] = -1;
            }
        }
        free(map);
    }
    /* exclusive scan (:2602), nnzC = last (:2604) */
    long long nnzc = 0;
    for (int t = 0; t < numblkC; t++) {
        int v = C->tile_nnz[t];
        C->tile_nnz[t] = (int)nnzc;
        nnzc += v;
        if (nnzc > 0x7fffffffLL) return -4;
    }
    C->tile_nnz[numblkC] = (int)nnzc;
    C->nnz = (int)nnzc;

    /* step 3: local columns from the masks, values accumulated at each
     * column's rank in its row (the row's Ptr + the mask bits before it) */
    C->tile_csr_Col = (uint16_t *)xcalloc((size_t)nnzc, sizeof(uint16_t));
    C->tile_csr_Value = (double *)xcalloc((size_t)nnzc, sizeof(double));
#pragma omp parallel
    {
        int *map = (int *)malloc(((size_t)blknB + 1) * sizeof(int));
        for (int j = 0; j < blknB; j++) map[j] = -1;
#pragma omp for schedule(dynamic, 2)
        for (int i = 0; i < blkmA; i++) {
            for (int t = C->tile_ptr[i]; t < C->tile_ptr[i + 1]; t++) {
                map[C->tile_columnidx[t]] = t;
                const uint16_t *mc = C->mask + (size_t)t * tm * wpr;
                int w = C->tile_nnz[t];
                for (int r = 0; r < tm; r++)
                    for (int x = 0; x < tm; x++)
                        if ((mc[r * wpr + x / MASK_BITS] >> (MASK_BITS - 1 - x % MASK_BITS)) & 1u)
                            C->tile_csr_Col[w++] = (uint16_t)x;
            }
            for (int a = A->tile_ptr[i]; a < A->tile_ptr[i + 1]; a++) {
                int k = A->tile_columnidx[a];
                for (int brm = B->tile_ptr[k]; brm < B->tile_ptr[k + 1]; brm++) {
                    int j = B->tile_columnidx[brm], t = map[j];
                    int b0 = B->csc_tile_ptr[j], b1 = B->csc_tile_ptr[j + 1];
                    int b = find_tile(B->csc_tile_rowidx, b0, b1, k);
                    const uint16_t *mc = C->mask + (size_t)t * tm * wpr;
                    const uint16_t *bp = B->tile_csr_Ptr + (size_t)b * tn;
                    int bnz0 = B->tile_nnz[b], bnz1 = B->tile_nnz[b + 1];
                    double *cv = C->tile_csr_Value + C->tile_nnz[t];
                    const uint16_t *cp = C->tile_csr_Ptr + (size_t)t * tm;
                    for (int q = A->tile_nnz[a]; q < A->tile_nnz[a + 1]; q++) {
                        int r = A->tile_csr_Col[q] / tn, c = A->tile_csr_Col[q] % tn;
                        double va = A->tile_csr_Value[q];
                        int s0 = bnz0 + bp[c], s1 = (c == tn - 1) ? bnz1 : bnz0 + bp[c + 1];
                        for (int s = s0; s < s1; s++) {
                            int x = B->tile_csr_Col[s], rk = cp[r];
                            for (int w = 0; w < x / MASK_BITS; w++) rk += __builtin_popcount(mc[r * wpr + w]);
                            int sh = MASK_BITS - x % MASK_BITS;  /* the bits of columns before x in its word */
                            rk += __builtin_popcount((unsigned)(mc[r * wpr + x / MASK_BITS] >> sh));
                            cv[rk] += va * B->tile_csr_Value[s];
                        }
                    }
                }
            }
            for (int t = C->tile_ptr[i]; t < C->tile_ptr[i + 1]; t++) map[C->tile_columnidx[t]] = -1;
        }
        free(map);
    }
    return 0;
}

/* tile2csr: src/tile2csr.h:72-140 (row counts from the per-tile Ptr, exclusive
 * scan, then per row the tiles in tile_ptr order; col = tile_col*tn + local). */
int tsgo_tile2csr(tsgo_mat *C, int tm, int tn) {
    int m = C->m;
    free(C->rowpointer); free(C->columnindex); free(C->value);
    int *rp = (int *)xcalloc((size_t)m + 1, sizeof(int));
    for (int i = 0; i < C->tilem; i++) {
        int rowlen = (i == C->tilem - 1) ? m - (C->tilem - 1) * tm : tm;
        for (int t = C->tile_ptr[i]; t < C->tile_ptr[i + 1]; t++) {
            int tnz = C->tile_nnz[t + 1] - C->tile_nnz[t];
            const uint16_t *p = C->tile_csr_Ptr + (size_t)t * tm;
            for (int r = 0; r < rowlen; r++) {
                int stop = (r == rowlen - 1) ? tnz : p[r + 1];
                rp[i * tm + r] += stop - p[r];
            }
        }
    }
    excl_scan_int(rp, (long)m + 1);
    int nnz = rp[m];
    int *ci = (int *)xcalloc(nnz, sizeof(int));
    double *cv = (double *)xcalloc(nnz, sizeof(double));
    int *fill = (int *)xcalloc((size_t)m + 1, sizeof(int));
    for (int i = 0; i < C->tilem; i++) {
        int rowlen = (i == C->tilem - 1) ? m - (C->tilem - 1) * tm : tm;
        for (int t = C->tile_ptr[i]; t < C->tile_ptr[i + 1]; t++) {
            int tnz = C->tile_nnz[t + 1] - C->tile_nnz[t], base = C->tile_nnz[t];
            const uint16_t *p = C->tile_csr_Ptr + (size_t)t * tm;
            for (int r = 0; r < rowlen; r++) {
                int stop = (r == rowlen - 1) ? tnz : p[r + 1];
                for (int q = p[r]; q < stop; q++) {
                    int R = i * tm + r, d = rp[R] + fill[R]++;
                    ci[d] = C->tile_columnidx[t] * tn + C->tile_csr_Col[base + q];
                    cv[d] = C->tile_csr_Value[base + q];
                }
            }
        }
    }
    free(fill);
    C->rowpointer = rp; C->columnindex = ci; C->value = cv; C->nnz = nnz;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* spgemm_spa: src/spgemm_serialref_spa_new.h:7-105.  Per thread a flag array of
 * nB/32+1 words, cleared for every row (:39,:70); count = popcount (:50-58);
 * fill emits set bits LSB-first per word = ascending columns (:84-99). */
int tsgo_spa(const tsgo_mat *A, const tsgo_mat *B, int *rowptrC, int *colidxC,
             long long *nnzC, int get_nnzC_only, int row_begin, int row_end) {
    int nB = B->n, words = nB / 32 + 1;
    int nth = tsgo_num_threads();
    unsigned *flags = (unsigned *)xcalloc((size_t)nth * words, sizeof(unsigned));
    if (!flags) return -1;
    if (row_begin < 0) row_begin = 0;
    if (row_end > A->m) row_end = A->m;
    if (get_nnzC_only) {
#pragma omp parallel for schedule(dynamic, 64)
        for (int i = row_begin; i < row_end; i++) {
            int tid = 0;
#ifdef _OPENMP
            tid = omp_get_thread_num();
#endif
            unsigned *fl = flags + (size_t)tid * words;
            memset(fl, 0, (size_t)words * sizeof(unsigned));
            for (int p = A->rowpointer[i]; p < A->rowpointer[i + 1]; p++) {
                int k = A->columnindex[p];
                for (int q = B->rowpointer[k]; q < B->rowpointer[k + 1]; q++) {
                    int key = B->columnindex[q];
                    fl[key >> 5] |= 1u << (key & 31);
                }
            }
            int c = 0;
            for (int w = 0; w < words; w++) c += __builtin_popcount(fl[w]);
            rowptrC[i] = c;
        }
        long long run = 0;
        for (int i = 0; i < row_begin; i++) rowptrC[i] = 0;
        for (int i = row_end; i <= A->m; i++) rowptrC[i] = 0;
        for (int i = 0; i <= A->m; i++) {
            long long v = rowptrC[i];
            rowptrC[i] = (int)run;
            run += v;
        }
        *nnzC = run;
        if (run > 0x7fffffffLL) {  /* past int32 row pointers (the reference's int nnzC) */
            free(flags);
            return -2;
        }
    } else {
#pragma omp parallel for schedule(dynamic, 64)
        for (int i = row_begin; i < row_end; i++) {
            int tid = 0;
#ifdef _OPENMP
            tid = omp_get_thread_num();
#endif
            unsigned *fl = flags + (size_t)tid * words;
            memset(fl, 0, (size_t)words * sizeof(unsigned));
            for (int p = A->rowpointer[i]; p < A->rowpointer[i + 1]; p++) {
                int k = A->columnindex[p];
                for (int q = B->rowpointer[k]; q < B->rowpointer[k + 1]; q++) {
                    int key = B->columnindex[q];
                    fl[key >> 5] |= 1u << (key & 31);
                }
            }
            int w0 = rowptrC[i];
            for (int w = 0; w < words; w++) {
                unsigned x = fl[w];
                while (x) {
                    int b = __builtin_ctz(x);
                    colidxC[w0++] = w * 32 + b;
                    x &= x - 1;
                }
            }
        }
    }
    free(flags);
    return 0;
}

/* Numeric dense-row SPA (src/external/cusparse/spgemm_serialref_spa.h:7-119),
 * parallelised over rows; the touched-column list replaces the O(nC) sweep. */
static int cmp_int(const void *a, const void *b) {
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

int tsgo_gustavson(const tsgo_mat *A, const tsgo_mat *B, tsgo_mat *C) {
    memset(C, 0, sizeof(*C));
    if (A->n != B->m) return -1;
    int m = A->m, n = B->n, nth = tsgo_num_threads();
    int *rp = (int *)xcalloc((size_t)m + 1, sizeof(int));
    char *flag = (char *)xcalloc((size_t)nth * n, 1);
    int *list = (int *)xcalloc((size_t)nth * n, sizeof(int));
#pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < m; i++) {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        char *fl = flag + (size_t)tid * n;
        int *ls = list + (size_t)tid * n, c = 0;
        for (int p = A->rowpointer[i]; p < A->rowpointer[i + 1]; p++) {
            int k = A->columnindex[p];
            for (int q = B->rowpointer[k]; q < B->rowpointer[k + 1]; q++) {
                int x = B->columnindex[q];
                if (!fl[x]) { fl[x] = 1; ls[c++] = x; }
            }
        }
        for (int u = 0; u < c; u++) fl[ls[u]] = 0;
        rp[i] = c;
    }
    long long run = 0;
    for (int i = 0; i <= m; i++) {
        long long v = rp[i];
        rp[i] = (int)run;
        run += v;
    }
    if (run > 0x7fffffffLL) { free(rp); free(flag); free(list); return -4; }
    int *ci = (int *)xcalloc((size_t)run, sizeof(int));
    double *cv = (double *)xcalloc((size_t)run, sizeof(double));
    double *acc = (double *)xcalloc((size_t)nth * n, sizeof(double));
#pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < m; i++) {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        char *fl = flag + (size_t)tid * n;
        int *ls = list + (size_t)tid * n, c = 0;
        double *ac = acc + (size_t)tid * n;
        for (int p = A->rowpointer[i]; p < A->rowpointer[i + 1]; p++) {
            int k = A->columnindex[p];
            double va = A->value[p];
            for (int q = B->rowpointer[k]; q < B->rowpointer[k + 1]; q++) {
                int x = B->columnindex[q];
                if (!fl[x]) { fl[x] = 1; ls[c++] = x; ac[x] = 0.0; }
                ac[x] += va * B->value[q];
            }
        }
        qsort(ls, (size_t)c, sizeof(int), cmp_int);
        for (int u = 0; u < c; u++) {
            ci[rp[i] + u] = ls[u];
            cv[rp[i] + u] = ac[ls[u]];
            fl[ls[u]] = 0;
        }
    }
    free(flag); free(list); free(acc);
    C->m = m; C->n = n; C->nnz = (int)run;
    C->rowpointer = rp; C->columnindex = ci; C->value = cv;
    return 0;
}

long long tsgo_gustavson_rows(const tsgo_mat *A, const tsgo_mat *B, int row_begin, int row_end) {
    int n = B->n, nth = tsgo_num_threads();
    if (row_begin < 0) row_begin = 0;
    if (row_end > A->m) row_end = A->m;
    char *flag = (char *)xcalloc((size_t)nth * n, 1);
    int *list = (int *)xcalloc((size_t)nth * n, sizeof(int));
    double *acc = (double *)xcalloc((size_t)nth * n, sizeof(double));
    long long total = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : total)
    for (int i = row_begin; i < row_end; i++) {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        char *fl = flag + (size_t)tid * n;
        int *ls = list + (size_t)tid * n, c = 0;
        double *ac = acc + (size_t)tid * n;
        for (int p = A->rowpointer[i]; p < A->rowpointer[i + 1]; p++) {
            int k = A->columnindex[p];
            double va = A->value[p];
            for (int q = B->rowpointer[k]; q < B->rowpointer[k + 1]; q++) {
                int x = B->columnindex[q];
                if (!fl[x]) { fl[x] = 1; ls[c++] = x; ac[x] = 0.0; }
                ac[x] += va * B->value[q];
            }
        }
        qsort(ls, (size_t)c, sizeof(int), cmp_int);
        for (int u = 0; u < c; u++) fl[ls[u]] = 0;
        total += c;
    }
    free(flag); free(list); free(acc);
    return total;
}

void tsgo_free(tsgo_mat *M) {
    if (!M) return;
    free(M->value); free(M->columnindex); free(M->rowpointer);
    free(M->tile_ptr); free(M->tile_columnidx); free(M->tile_rowidx); free(M->tile_nnz);
    free(M->tile_csr_Value); free(M->tile_csr_Col); free(M->tile_csr_Ptr); free(M->mask);
    free(M->csc_tile_ptr); free(M->csc_tile_rowidx);
    memset(M, 0, sizeof(*M));
}
