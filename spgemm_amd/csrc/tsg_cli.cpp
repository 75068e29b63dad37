// tsg_cli.cpp -- the reference's `./test -d <dev> -aat <0|1> <A.mtx> [tile_m tile_n]`
// driver (src/main.cu:13-359) on top of libtsg.so.  Same flow and key output
// lines; tile sizes default to 16 16 (the upstream 4-argument form,
// data/run18.sh:12).  CSV rows go to $TSG_DATA_DIR (default ../data), which is
// created when missing instead of crashing (src/main.cu:283-320).
#include <sys/stat.h>
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/tsg.h"

static double now_ms() {
    timeval t;
    gettimeofday(&t, nullptr);
    return t.tv_sec * 1000.0 + t.tv_usec / 1000.0;
}

static FILE *open_csv(const std::string &dir, const char *name) {
    mkdir(dir.c_str(), 0755);
    std::string p = dir + "/" + name;
    FILE *f = fopen(p.c_str(), "a");
    if (!f) printf("Writing results fails (%s).\n", p.c_str());
    return f;
}

int main(int argc, char **argv) {
    // the reference prints each step's time: the step markers on (the library
    // records them only on request; an explicit TSG_STAGE_EVENTS=0 wins)
    setenv("TSG_STAGE_EVENTS", "1", 0);
    if (argc < 6) {
        printf("Run the code by './test -d 0 -aat 0 matrix.mtx tile_size_m tile_size_n'.\n");
        return 0;
    }
    printf("--------------------------------!!!!!!!!------------------------------------\n");
    int argi = 1;
    if (strcmp(argv[argi], "-d") != 0) return 0;
    int device_id = atoi(argv[argi + 1]);
    argi += 2;
    printf("device_id = %i\n", device_id);
    int ndev = 0;
    tsg_device_count(&ndev);
    if (ndev <= 0) {
        fprintf(stderr, "tsg: no HIP device visible (%s)\n", tsg_status_string(TSG_ERR_NO_DEVICE));
        return 1;
    }
    if (strcmp(argv[argi], "-aat") != 0) return 0;
    int aat = atoi(argv[argi + 1]);
    argi += 2;
    const char *filename = argv[argi++];
    int tm = argi < argc ? atoi(argv[argi++]) : 16;
    int tn = argi < argc ? atoi(argv[argi++]) : 16;
    printf("---------------------------------------------------------------\n");
    printf("Device [ %i ] %s\n", device_id, tsg_version());
    printf("MAT: -------------- %s --------------\n", filename);

    tsg_smatrix A{}, B{}, C{};
    double t1 = now_ms();
    int rc = tsg_mmio_allinone(filename, &A);
    double tload = now_ms() - t1;
    if (rc != TSG_OK) {
        fprintf(stderr, "tsg: cannot read %s: %s\n", filename, tsg_status_string(rc));
        return 1;
    }
    printf("input matrix A: ( %i, %i ) nnz = %i\n loadfile time    = %4.5f sec\n", A.m, A.n, A.nnz, tload / 1000.0);
    if (!aat && A.m != A.n) {
        printf("matrix squaring must have rowA == colA. Exit.\n");
        return 0;
    }
    printf("the tile_size_m = %d\n", tm);
    printf("the tile_size_n = %d\n", tn);
    tsg_values_pos_mod10(&A);
    bool alias = false;
    if (aat) {
        if (A.m == A.n && A.isSymmetric) {
            printf("matrix AAT does not do symmetric matrix. Exit.\n");
            return 0;
        }
        if ((rc = tsg_transpose(&A, &B)) != TSG_OK) {
            fprintf(stderr, "tsg: transpose failed: %s\n", tsg_status_string(rc));
            return 1;
        }
    } else {
        B.m = A.m; B.n = A.n; B.nnz = A.nnz;
        B.rowpointer = A.rowpointer; B.columnindex = A.columnindex; B.value = A.value;
        alias = true;
    }
    unsigned long long nnzCub = 0;
    if ((rc = tsg_nnzcub(&A, &B, &nnzCub)) != TSG_OK) {
        fprintf(stderr, "tsg: nnzCub failed: %s\n", tsg_status_string(rc));
        return 1;
    }
    printf("SpGEMM nnzCub = %lld\n", (long long)nnzCub);

    t1 = now_ms();
    rc = tsg_csr2tile_row_major(&A, tm, tn);
    double time_conversion = now_ms() - t1;
    if (rc != TSG_OK) {
        fprintf(stderr, "tsg: csr2tile_row_major failed: %s\n", tsg_status_string(rc));
        return 1;
    }
    printf("CSR to Tile conversion uses %.2f ms\n", time_conversion);
    double tile_bytes = (A.tilem + 1) * 4.0 + A.numtile * 4.0 + (A.numtile + 1) * 4.0 + A.nnz * 8.0 + A.nnz * 1.0 +
                        A.numtile * 16.0 * 1.0 + A.numtile * 16.0 * 2.0;  // src/main.cu:178-180
    double mem = tile_bytes / 1024 / 1024;
    double csr_mem = ((A.m + 1) * 4.0 + A.nnz * 4.0 + A.nnz * 8.0) / 1024 / 1024;
    printf("tile space overhead = %.2f MB\n", mem);
    if ((rc = tsg_csr2tile_col_major(&B, tm, tn)) != TSG_OK) {
        fprintf(stderr, "tsg: csr2tile_col_major failed: %s\n", tsg_status_string(rc));
        return 1;
    }
    unsigned long long nnzC = 0;
    double compression = 0, time_tile = 0, gflops = 0, ts1 = 0, ts2 = 0, ts3 = 0, tmal = 0;
    rc = tsg_tilespgemm(&A, &B, &C, nullptr, nullptr, 0, 0.0, 0.0, nnzCub, &nnzC, &compression, &time_tile, &gflops,
                        filename, &ts1, &ts2, &ts3, &tmal, tm, tn);
    if (rc != TSG_OK) {
        fprintf(stderr, "tsg: tilespgemm failed: %s\n", tsg_status_string(rc));
        return 1;
    }
    const char *dd = getenv("TSG_DATA_DIR");
    std::string dir = dd ? dd : "../data";
    if (FILE *f = open_csv(dir, "results_tile.csv")) {
        fprintf(f, "%s,%i,%i,%i,%lld,%lld,%f,%f,%f\n", filename, A.m, A.n, A.nnz, (long long)nnzCub, (long long)nnzC,
                compression, time_tile, gflops);
        fclose(f);
    }
    if (FILE *f = open_csv(dir, "step_runtime.csv")) {
        fprintf(f, "%s,%i,%i,%i,%lld,%lld,%f,%f,%f,%f,%f\n", filename, A.m, A.n, A.nnz, (long long)nnzCub,
                (long long)nnzC, compression, ts1, ts2, ts3, tmal);
        fclose(f);
    }
    if (FILE *f = open_csv(dir, "mem-cost.csv")) {
        fprintf(f, "%s,%i,%i,%i,%lld,%lld,%f,%f,%f\n", filename, A.m, A.n, A.nnz, (long long)nnzCub, (long long)nnzC,
                compression, csr_mem, mem);
        fclose(f);
    }
    if (FILE *f = open_csv(dir, "preprocessing.csv")) {
        fprintf(f, "%s,%i,%i,%i,%lld,%lld,%f,%f,%f\n", filename, A.m, A.n, A.nnz, (long long)nnzCub, (long long)nnzC,
                compression, time_conversion, time_tile);
        fclose(f);
    }
    printf("-------------------------------check----------------------------------------\n");
    if ((rc = tsg_tile2csr(&C, tm, tm)) != TSG_OK) {
        fprintf(stderr, "tsg: tile2csr failed: %s\n", tsg_status_string(rc));
        return 1;
    }
    printf("tile to CSR conversion complete!\n");
    printf("nnzC (CSR) = %i\n", C.nnz);
    printf("---------------------------------------------------------------\n");
    tsg_matrix_destroy(&C);
    if (alias) {
        B.rowpointer = nullptr; B.columnindex = nullptr; B.value = nullptr;
    }
    tsg_matrix_destroy(&B);
    tsg_matrix_destroy(&A);
    return 0;
}
