// Test infrastructure only: an independent on-GPU SpGEMM (rocSPARSE) used to
// cross-check libtsg's C at sizes where the CPU oracle is slow (SURVEY.md §8f
// rank 2, mirroring the reference's cuSPARSE check src/spgemm_cu.h:5-41).
// Host CSR in, host CSR out (malloc'd; free with rs_free).  Not part of the product.
#include <hip/hip_runtime.h>
#include <rocsparse/rocsparse.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK_HIP(x)                                                                 \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "rs_spgemm: %s: %s\n", #x, hipGetErrorString(e_));    \
            return -2;                                                            \
        }                                                                         \
    } while (0)
#define CK_RS(x)                                                                  \
    do {                                                                          \
        rocsparse_status s_ = (x);                                                \
        if (s_ != rocsparse_status_success) {                                     \
            fprintf(stderr, "rs_spgemm: %s: status %d\n", #x, (int)s_);          \
            return -3;                                                            \
        }                                                                         \
    } while (0)

template <class T> static int up(T **d, const T *h, size_t n) {
    CK_HIP(hipMalloc((void **)d, (n ? n : 1) * sizeof(T)));
    if (n) CK_HIP(hipMemcpy(*d, h, n * sizeof(T), hipMemcpyHostToDevice));
    return 0;
}

static double g_last_ms = 0.0;  // device time of the last call's three stages (diagnostics)
extern "C" double rs_last_ms() { return g_last_ms; }

extern "C" int rs_spgemm(int m, int k, int n, int nnzA, const int *rpA, const int *ciA, const double *vA, int nnzB,
                         const int *rpB, const int *ciB, const double *vB, long long *nnzC_out, int **rpC,
                         int **ciC, double **vC) {
    int *dA_rp, *dA_ci, *dB_rp, *dB_ci, *dC_rp, *dC_ci = nullptr;
    double *dA_v, *dB_v, *dC_v = nullptr;
    if (up(&dA_rp, rpA, (size_t)m + 1) || up(&dA_ci, ciA, nnzA) || up(&dA_v, vA, nnzA)) return -2;
    if (up(&dB_rp, rpB, (size_t)k + 1) || up(&dB_ci, ciB, nnzB) || up(&dB_v, vB, nnzB)) return -2;
    CK_HIP(hipMalloc((void **)&dC_rp, ((size_t)m + 1) * sizeof(int)));
    rocsparse_handle h;
    CK_RS(rocsparse_create_handle(&h));
    rocsparse_spmat_descr A, B, C;
    const rocsparse_indextype i32 = rocsparse_indextype_i32;
    const rocsparse_index_base b0 = rocsparse_index_base_zero;
    const rocsparse_datatype f64 = rocsparse_datatype_f64_r;
    CK_RS(rocsparse_create_csr_descr(&A, m, k, nnzA, dA_rp, dA_ci, dA_v, i32, i32, b0, f64));
    CK_RS(rocsparse_create_csr_descr(&B, k, n, nnzB, dB_rp, dB_ci, dB_v, i32, i32, b0, f64));
    CK_RS(rocsparse_create_csr_descr(&C, m, n, 0, dC_rp, nullptr, nullptr, i32, i32, b0, f64));
    // D: an empty m x n matrix (beta = 0); rocSPARSE wants a valid descriptor
    int *dD_rp;
    CK_HIP(hipMalloc((void **)&dD_rp, ((size_t)m + 1) * sizeof(int)));
    CK_HIP(hipMemset(dD_rp, 0, ((size_t)m + 1) * sizeof(int)));
    rocsparse_spmat_descr D;
    CK_RS(rocsparse_create_csr_descr(&D, m, n, 0, dD_rp, nullptr, nullptr, i32, i32, b0, f64));
    const double alpha = 1.0, beta = 0.0;
    const rocsparse_operation nt = rocsparse_operation_none;
    size_t bsz = 0;
    void *buf = nullptr;
    hipEvent_t e0, e1;
    CK_HIP(hipEventCreate(&e0));
    CK_HIP(hipEventCreate(&e1));
    CK_HIP(hipEventRecord(e0, 0));
    CK_RS(rocsparse_spgemm(h, nt, nt, &alpha, A, B, &beta, D, C, f64, rocsparse_spgemm_alg_default,
                           rocsparse_spgemm_stage_buffer_size, &bsz, nullptr));
    CK_HIP(hipMalloc(&buf, bsz ? bsz : 1));
    CK_RS(rocsparse_spgemm(h, nt, nt, &alpha, A, B, &beta, D, C, f64, rocsparse_spgemm_alg_default,
                           rocsparse_spgemm_stage_nnz, &bsz, buf));
    int64_t rows, cols, nnzC;
    CK_RS(rocsparse_spmat_get_size(C, &rows, &cols, &nnzC));
    CK_HIP(hipMalloc((void **)&dC_ci, (nnzC ? nnzC : 1) * sizeof(int)));
    CK_HIP(hipMalloc((void **)&dC_v, (nnzC ? nnzC : 1) * sizeof(double)));
    CK_RS(rocsparse_csr_set_pointers(C, dC_rp, dC_ci, dC_v));
    CK_RS(rocsparse_spgemm(h, nt, nt, &alpha, A, B, &beta, D, C, f64, rocsparse_spgemm_alg_default,
                           rocsparse_spgemm_stage_compute, &bsz, buf));
    CK_HIP(hipEventRecord(e1, 0));
    CK_HIP(hipDeviceSynchronize());
    float ms = 0.f;
    CK_HIP(hipEventElapsedTime(&ms, e0, e1));
    g_last_ms = ms;  // includes rocSPARSE's buffer/C allocations, as the stages need them
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    *nnzC_out = nnzC;
    *rpC = (int *)malloc(((size_t)m + 1) * sizeof(int));
    *ciC = (int *)malloc((nnzC ? nnzC : 1) * sizeof(int));
    *vC = (double *)malloc((nnzC ? nnzC : 1) * sizeof(double));
    CK_HIP(hipMemcpy(*rpC, dC_rp, ((size_t)m + 1) * sizeof(int), hipMemcpyDeviceToHost));
    if (nnzC) {
        CK_HIP(hipMemcpy(*ciC, dC_ci, nnzC * sizeof(int), hipMemcpyDeviceToHost));
        CK_HIP(hipMemcpy(*vC, dC_v, nnzC * sizeof(double), hipMemcpyDeviceToHost));
    }
    rocsparse_destroy_spmat_descr(A);
    rocsparse_destroy_spmat_descr(B);
    rocsparse_destroy_spmat_descr(C);
    rocsparse_destroy_spmat_descr(D);
    hipFree(dD_rp);
    rocsparse_destroy_handle(h);
    hipFree(buf);
    hipFree(dA_rp); hipFree(dA_ci); hipFree(dA_v);
    hipFree(dB_rp); hipFree(dB_ci); hipFree(dB_v);
    hipFree(dC_rp); hipFree(dC_ci); hipFree(dC_v);
    return 0;
}

extern "C" void rs_free(void *p) { free(p); }
