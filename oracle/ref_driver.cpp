// ref_driver.cpp -- builds oracle/_ref/ref_driver from the reference's OWN host
// sources where they lie (/root/reference/src, included read-only through -I).
// TEST INFRASTRUCTURE ONLY: used to generate tests/golden/ fixtures that pin the
// oracle restatement (oracle/tsg_oracle.c).  Never shipped, never run on the GPU box.
//
// Usage: ref_driver <A.mtx> <aat 0|1> <tile_m> <tile_n> <out.bin>
// Mirrors the host-side flow of src/main.cu:97-191 (load, value overwrite,
// optional transpose, nnzCub, csr2tile_row_major(A), csr2tile_col_major(B)),
// then records spgemm_spa(A,B) (src/spgemm_serialref_spa_new.h) for the C
// pattern and spgemm_spa over the two tile patterns for the C tile structure.
#include <cassert>
#include "common.h"
#include "mmio_highlevel.h"
#include "utils.h"
#include "csr2tile.h"
#include "tile2csr.h"
#include "spgemm_serialref_spa_new.h"

#include <cstdio>
#include <cstring>
#include <cstdint>
#include <string>

static FILE *g_out;

static void rec(const char *name, char code, const void *p, uint64_t count, size_t esz) {
    uint32_t nl = (uint32_t)strlen(name);
    fwrite(&nl, 4, 1, g_out);
    fwrite(name, 1, nl, g_out);
    fwrite(&code, 1, 1, g_out);
    fwrite(&count, 8, 1, g_out);
    if (count) fwrite(p, esz, count, g_out);
}
static void rec_i(const char *n, const int *p, uint64_t c) { rec(n, 'i', p, c, 4); }
static void rec_h(const char *n, const uint16_t *p, uint64_t c) { rec(n, 'h', p, c, 2); }
static void rec_d(const char *n, const double *p, uint64_t c) { rec(n, 'd', p, c, 8); }
static void rec_scalar(const char *n, long long v) { rec(n, 'q', &v, 1, 8); }

static void dump_csr(const char *pfx, SMatrix *M) {
    std::string s(pfx);
    rec_scalar((s + ".m").c_str(), M->m);
    rec_scalar((s + ".n").c_str(), M->n);
    rec_scalar((s + ".nnz").c_str(), M->nnz);
    rec_i((s + ".rowpointer").c_str(), M->rowpointer, (uint64_t)M->m + 1);
    rec_i((s + ".columnindex").c_str(), M->columnindex, (uint64_t)M->nnz);
    rec_d((s + ".value").c_str(), M->value, (uint64_t)M->nnz);
}

static void dump_tiles(const char *pfx, SMatrix *M, int ptr_rows, int mask_words, bool csc) {
    std::string s(pfx);
    rec_scalar((s + ".tilem").c_str(), M->tilem);
    rec_scalar((s + ".tilen").c_str(), M->tilen);
    rec_scalar((s + ".numtile").c_str(), M->numtile);
    rec_i((s + ".tile_ptr").c_str(), M->tile_ptr, (uint64_t)M->tilem + 1);
    rec_i((s + ".tile_columnidx").c_str(), M->tile_columnidx, (uint64_t)M->numtile);
    rec_i((s + ".tile_nnz").c_str(), M->tile_nnz, (uint64_t)M->numtile + 1);
    rec_h((s + ".tile_csr_Ptr").c_str(), M->tile_csr_Ptr, (uint64_t)M->numtile * ptr_rows);
    rec_h((s + ".tile_csr_Col").c_str(), M->tile_csr_Col, (uint64_t)M->nnz);
    rec_d((s + ".tile_csr_Value").c_str(), M->tile_csr_Value, (uint64_t)M->nnz);
    rec_h((s + ".mask").c_str(), M->mask, (uint64_t)M->numtile * ptr_rows * mask_words);
    if (csc) {
        rec_i((s + ".csc_tile_ptr").c_str(), M->csc_tile_ptr, (uint64_t)M->tilen + 1);
        rec_i((s + ".csc_tile_rowidx").c_str(), M->csc_tile_rowidx, (uint64_t)M->numtile);
    }
}

int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: ref_driver A.mtx aat tm tn out.bin\n");
        return 2;
    }
    int aat = atoi(argv[2]), tm = atoi(argv[3]), tn = atoi(argv[4]);
    SMatrix *A = (SMatrix *)calloc(1, sizeof(SMatrix));
    SMatrix *B = (SMatrix *)calloc(1, sizeof(SMatrix));
    if (mmio_allinone(&A->m, &A->n, &A->nnz, &A->isSymmetric, &A->rowpointer,
                      &A->columnindex, &A->value, argv[1]) != 0) {
        fprintf(stderr, "load failed\n");
        return 3;
    }
    for (int i = 0; i < A->nnz; i++) A->value[i] = i % 10;
    if (aat) {
        B->m = A->n; B->n = A->m; B->nnz = A->nnz;
        B->rowpointer = (int *)malloc((A->n + 1) * sizeof(int));
        B->columnindex = (int *)malloc(A->nnz * sizeof(int));
        B->value = (double *)malloc(A->nnz * sizeof(double));
        matrix_transposition(A->m, A->n, A->nnz, A->rowpointer, A->columnindex, A->value,
                             B->columnindex, B->rowpointer, B->value);
    } else {
        B->m = A->m; B->n = A->n; B->nnz = A->nnz;
        B->rowpointer = A->rowpointer; B->columnindex = A->columnindex; B->value = A->value;
    }
    g_out = fopen(argv[5], "wb");
    if (!g_out) return 4;
    dump_csr("A", A);
    dump_csr("B", B);
    unsigned long long nnzCub = 0;
    for (int i = 0; i < A->nnz; i++) {
        int r = A->columnindex[i];
        nnzCub += B->rowpointer[r + 1] - B->rowpointer[r];
    }
    rec_scalar("nnzCub", (long long)nnzCub);

    // element-level C pattern through the reference's CPU SPA
    int *rpC = (int *)calloc(A->m + 1, sizeof(int));
    int nnzC = 0;
    spgemm_spa(A->rowpointer, A->columnindex, A->value, A->m, A->n, A->nnz,
               B->rowpointer, B->columnindex, B->value, B->m, B->n, B->nnz,
               rpC, NULL, NULL, A->m, B->n, &nnzC, 1);
    int *ciC = (int *)calloc(nnzC > 0 ? nnzC : 1, sizeof(int));
    spgemm_spa(A->rowpointer, A->columnindex, A->value, A->m, A->n, A->nnz,
               B->rowpointer, B->columnindex, B->value, B->m, B->n, B->nnz,
               rpC, ciC, NULL, A->m, B->n, &nnzC, 0);
    rec_i("C.rowpointer", rpC, (uint64_t)A->m + 1);
    rec_i("C.columnindex", ciC, (uint64_t)nnzC);

    csr2tile_row_major(A, tm, tn);
    csr2tile_col_major(B, tm, tn);
    dump_tiles("At", A, tm, tn / 16, false);
    dump_tiles("Bt", B, tn, tm / 16, true);

    // C tile structure = SPA over the tile patterns (what step 1 computes)
    int *rpCt = (int *)calloc(A->tilem + 1, sizeof(int));
    int numblkC = 0;
    spgemm_spa(A->tile_ptr, A->tile_columnidx, NULL, A->tilem, A->tilen, A->numtile,
               B->tile_ptr, B->tile_columnidx, NULL, B->tilem, B->tilen, B->numtile,
               rpCt, NULL, NULL, A->tilem, B->tilen, &numblkC, 1);
    int *ciCt = (int *)calloc(numblkC > 0 ? numblkC : 1, sizeof(int));
    spgemm_spa(A->tile_ptr, A->tile_columnidx, NULL, A->tilem, A->tilen, A->numtile,
               B->tile_ptr, B->tile_columnidx, NULL, B->tilem, B->tilen, B->numtile,
               rpCt, ciCt, NULL, A->tilem, B->tilen, &numblkC, 0);
    rec_i("Ct.tile_ptr", rpCt, (uint64_t)A->tilem + 1);
    rec_i("Ct.tile_columnidx", ciCt, (uint64_t)numblkC);
    fclose(g_out);
    return 0;
}
