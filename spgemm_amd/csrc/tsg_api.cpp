// tsg_api.cpp -- C ABI of libtsg.so (include/tsg.h): context + caching device
// allocator, the reference-named host functions, and the Matrix-Market reader.
// All arithmetic of the hot path runs in the HIP kernels of tsg_device.hip; the
// host functions only move data and orchestrate.
#include <hip/hip_runtime.h>

#include <sys/stat.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "tsg_internal.h"

namespace tsg {
int dev_tiles_finalize_c(Context &cx, tsg_dev_tiles &C, hipStream_t s, bool zero_empty);
int dev_rm2csc_from_structs(Context &cx, tsg_dev_tiles &B, hipStream_t s);

void report_hip_error(hipError_t e, const char *what, const char *file, int line) {
    if (!getenv("TSG_QUIET_ERRORS"))
        fprintf(stderr, "[tsg] HIP error %d (%s) at %s:%d: %s\n", (int)e, hipGetErrorString(e), file, line, what);
}

// ------------------------------------------------------------------ pool
static size_t size_class(size_t b) {
    size_t c = 256;
    while (c < b) c <<= 1;
    return c;
}

DevicePool::~DevicePool() { trim(); }

int DevicePool::alloc(void **p, size_t bytes) {
    size_t c = size_class(bytes ? bytes : 1);
    auto it = free_.find(c);
    if (it != free_.end()) {
        *p = it->second;
        free_.erase(it);
        live_[*p] = c;
        return TSG_OK;
    }
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, c);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        trim();  // give cached blocks back and retry once
        e = hipMalloc(&q, c);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            *p = nullptr;
            return TSG_ERR_OOM;
        }
    }
    reserved_ += c;
    live_[q] = c;
    *p = q;
    return TSG_OK;
}

void DevicePool::release(void *p) {
    auto it = live_.find(p);
    if (it == live_.end()) return;
    free_.emplace(it->second, p);
    live_.erase(it);
}

void DevicePool::release_all_live() {
    for (auto &kv : live_) free_.emplace(kv.second, kv.first);
    live_.clear();
}

void DevicePool::trim() {
    for (auto &kv : free_) {
        (void)hipFree(kv.second);
        reserved_ -= kv.first;
    }
    free_.clear();
}

int Context::init(int dev) {
    device = dev;
    TSG_HIP(hipSetDevice(dev));
    TSG_HIP(hipHostMalloc((void **)&pinned, 64, hipHostMallocDefault));
    TSG_HIP(hipHostMalloc((void **)&pinned64, 256, hipHostMallocDefault));
    TSG_HIP(hipHostGetDevicePointer((void **)&dpinned, pinned, 0));
    TSG_HIP(hipHostGetDevicePointer((void **)&dpinned64, pinned64, 0));
    for (auto &e : ev) TSG_HIP(hipEventCreate(&e));
    ev_ready = true;
    return TSG_OK;
}

int stream_wait(hipStream_t s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return TSG_OK;
        if (e != hipErrorNotReady) {
            report_hip_error(e, "hipStreamQuery", __FILE__, __LINE__);
            return TSG_ERR_HIP;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(1000)) break;
        std::this_thread::yield();  // (concurrent callers on other threads keep their cores)
    }
    TSG_HIP(hipStreamSynchronize(s));
    return TSG_OK;
}

void Context::destroy() {
    (void)hipSetDevice(device);
    (void)hipDeviceSynchronize();
    pool.release_all_live();
    pool.trim();
    if (pinned) (void)hipHostFree(pinned);
    if (pinned64) (void)hipHostFree(pinned64);
    pinned = nullptr;
    pinned64 = nullptr;
    if (ev_ready)
        for (auto &e : ev) (void)hipEventDestroy(e);
    ev_ready = false;
}

static double ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
        (void)hipGetLastError();
        return 0.0;
    }
    return (double)ms;
}

}  // namespace tsg

using namespace tsg;

struct tsg_context {
    Context cx;
    hipStream_t stream = nullptr;  // host-layer leases only (tsg_dev_* take the caller's stream)
};

// ------------------------------------------------------------------ helpers
static int g_have_device = -1;

static int check_device() {
    if (g_have_device < 0) {
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        if (e != hipSuccess) (void)hipGetLastError();
        g_have_device = (e == hipSuccess && n > 0) ? 1 : 0;
    }
    return g_have_device ? TSG_OK : TSG_ERR_NO_DEVICE;
}

// Host-layer (reference-named) calls: each call leases a context of the calling
// thread's current device from a per-device pool (mutex-guarded) and runs on that
// context's own non-blocking stream, so concurrent host threads never share a
// context, a stream or an allocator, and each call lands on the device the
// thread selected (SURVEY.md §8b "Threading").  Leased contexts are kept for
// reuse (their caches make repeated calls allocation-free).
struct HostPools {
    std::mutex mu;
    std::map<int, std::vector<tsg_context *>> idle;
};
static HostPools &host_pools() {
    static HostPools *p = new HostPools();  // never destroyed: safe at exit
    return *p;
}

class HostLease {
  public:
    HostLease() = default;
    HostLease(const HostLease &) = delete;
    HostLease &operator=(const HostLease &) = delete;
    int acquire() {
        TSG_TRY(check_device());
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) {
            (void)hipGetLastError();
            dev = 0;
        }
        {
            std::lock_guard<std::mutex> g(host_pools().mu);
            auto &v = host_pools().idle[dev];
            if (!v.empty()) {
                c_ = v.back();
                v.pop_back();
            }
        }
        if (!c_) {
            tsg_context *c = new tsg_context();
            int rc = c->cx.init(dev);
            if (rc == TSG_OK && hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
                (void)hipGetLastError();
                rc = TSG_ERR_HIP;
            }
            if (rc != TSG_OK) {
                c->cx.destroy();
                delete c;
                return rc;
            }
            c_ = c;
        }
        return TSG_OK;
    }
    ~HostLease() {
        if (!c_) return;
        (void)hipStreamSynchronize(c_->stream);
        c_->cx.pool.release_all_live();
        std::lock_guard<std::mutex> g(host_pools().mu);
        host_pools().idle[c_->cx.device].push_back(c_);
    }
    tsg_context *ctx() { return c_; }
    Context &cx() { return c_->cx; }
    hipStream_t stream() { return c_->stream; }

  private:
    tsg_context *c_ = nullptr;
};

template <class T> static int upload(Context &cx, T **d, const T *h, size_t n, hipStream_t s) {
    TSG_TRY(cx.get(d, n ? n : 1));
    if (n) TSG_HIP(hipMemcpyAsync(*d, h, n * sizeof(T), hipMemcpyHostToDevice, s));
    return TSG_OK;
}

template <class T> static int download(T **h, const T *d, size_t n, hipStream_t s) {
    *h = (T *)malloc((n ? n : 1) * sizeof(T));
    if (!*h) return TSG_ERR_OOM;
    if (n) TSG_HIP(hipMemcpyAsync(*h, d, n * sizeof(T), hipMemcpyDeviceToHost, s));
    return TSG_OK;
}

static bool valid_tiles(int tm, int tn) {
    return tm > 0 && tn > 0 && tm % 16 == 0 && tn % 16 == 0 && tm <= 64 && tn <= 64 && (long)tm * tn <= 65536;
}

static int upload_csr(Context &cx, const tsg_smatrix *A, tsg_dev_csr &d, hipStream_t s) {
    d.m = A->m;
    d.n = A->n;
    d.nnz = A->nnz;
    TSG_TRY(upload(cx, &d.rowpointer, A->rowpointer, (size_t)A->m + 1, s));
    TSG_TRY(upload(cx, &d.columnindex, A->columnindex, (size_t)A->nnz, s));
    TSG_TRY(upload(cx, &d.value, A->value, (size_t)A->nnz, s));
    return TSG_OK;
}

static void free_tile_fields(tsg_smatrix *M) {
    free(M->tile_ptr); free(M->tile_columnidx); free(M->tile_rowidx); free(M->tile_nnz);
    free(M->tile_csr_Value); free(M->tile_csr_Col); free(M->tile_csr_Ptr); free(M->mask);
    free(M->csc_tile_ptr); free(M->csc_tile_rowidx);
    M->tile_ptr = M->tile_columnidx = M->tile_rowidx = M->tile_nnz = nullptr;
    M->tile_csr_Value = nullptr;
    M->tile_csr_Col = M->tile_csr_Ptr = M->mask = nullptr;
    M->csc_tile_ptr = M->csc_tile_rowidx = nullptr;
}

static int download_tiles(const tsg_dev_tiles &t, tsg_smatrix *M, bool csc, hipStream_t s) {
    free_tile_fields(M);
    const size_t nt = (size_t)t.numtile;
    M->tilem = t.tilem;
    M->tilen = t.tilen;
    M->numtile = t.numtile;
    TSG_TRY(download(&M->tile_ptr, t.tile_ptr, (size_t)t.tilem + 1, s));
    TSG_TRY(download(&M->tile_columnidx, t.tile_columnidx, nt, s));
    if (t.tile_rowidx) TSG_TRY(download(&M->tile_rowidx, t.tile_rowidx, nt, s));
    TSG_TRY(download(&M->tile_nnz, t.tile_nnz, nt + 1, s));
    TSG_TRY(download(&M->tile_csr_Ptr, t.tile_csr_Ptr, nt * t.tile_m, s));
    TSG_TRY(download(&M->tile_csr_Col, t.tile_csr_Col, (size_t)t.nnz, s));
    TSG_TRY(download(&M->tile_csr_Value, t.tile_csr_Value, (size_t)t.nnz, s));
    if (t.mask) TSG_TRY(download(&M->mask, t.mask, nt * t.tile_m * (t.tile_n / 16), s));
    if (csc) {
        TSG_TRY(download(&M->csc_tile_ptr, t.csc_tile_ptr, (size_t)t.tilen + 1, s));
        TSG_TRY(download(&M->csc_tile_rowidx, t.csc_tile_rowidx, nt, s));
    }
    TSG_HIP(hipStreamSynchronize(s));
    return TSG_OK;
}

// the tile structure alone (tile_ptr, tile_columnidx): what step 1 reads
static int upload_tile_structure(Context &cx, const tsg_smatrix *M, int tile_m, int tile_n, tsg_dev_tiles &t,
                                 hipStream_t s) {
    t = tsg_dev_tiles{};
    t.m = M->m; t.n = M->n; t.nnz = M->nnz;
    t.tile_m = tile_m; t.tile_n = tile_n;
    t.tilem = M->tilem; t.tilen = M->tilen; t.numtile = M->numtile;
    TSG_TRY(upload(cx, &t.tile_ptr, M->tile_ptr, (size_t)M->tilem + 1, s));
    TSG_TRY(upload(cx, &t.tile_columnidx, M->tile_columnidx, (size_t)M->numtile, s));
    return TSG_OK;
}

static int upload_tiles(Context &cx, const tsg_smatrix *M, int tile_m, int tile_n, bool csc, tsg_dev_tiles &t,
                        hipStream_t s) {
    t = tsg_dev_tiles{};
    t.m = M->m; t.n = M->n; t.nnz = M->nnz;
    t.tile_m = tile_m; t.tile_n = tile_n;
    t.tilem = M->tilem; t.tilen = M->tilen; t.numtile = M->numtile;
    const size_t nt = (size_t)M->numtile;
    TSG_TRY(upload(cx, &t.tile_ptr, M->tile_ptr, (size_t)M->tilem + 1, s));
    TSG_TRY(upload(cx, &t.tile_columnidx, M->tile_columnidx, nt, s));
    TSG_TRY(upload(cx, &t.tile_nnz, M->tile_nnz, nt + 1, s));
    TSG_TRY(upload(cx, &t.tile_csr_Ptr, M->tile_csr_Ptr, nt * tile_m, s));
    TSG_TRY(upload(cx, &t.tile_csr_Col, M->tile_csr_Col, (size_t)M->nnz, s));
    TSG_TRY(upload(cx, &t.tile_csr_Value, M->tile_csr_Value, (size_t)M->nnz, s));
    if (M->mask) TSG_TRY(upload(cx, &t.mask, M->mask, nt * tile_m * (tile_n / 16), s));
    if (csc) {
        if (!M->csc_tile_ptr || !M->csc_tile_rowidx) return TSG_ERR_INVALID;
        TSG_TRY(upload(cx, &t.csc_tile_ptr, M->csc_tile_ptr, (size_t)M->tilen + 1, s));
        TSG_TRY(upload(cx, &t.csc_tile_rowidx, M->csc_tile_rowidx, nt, s));
        TSG_TRY(dev_rm2csc_from_structs(cx, t, s));
    }
    return TSG_OK;
}

// Step 2 streams element products when A averages fewer nonzeros per tile than
// this (one 16-bit row-mask OR per A nonzero and B tile otherwise wins).
static constexpr double kStep2ElemMaxTileDensity = 16.0;

static bool quiet() { return getenv("TSG_QUIET") != nullptr; }
// b_sorted: 1 = the caller already checked B's rows column-sorted (the check
// is skipped), -1 = unknown (checked here)
static int dev_spgemm16(Context &cx, const tsg_dev_csr *A, const tsg_dev_csr *B, hipStream_t s, tsg_dev_csr *C,
                        tsg_stats *stats, int b_sorted = -1);

// tsg_tilespgemm's CSR route computes C from the CSR that the reference's
// SMatrix carries beside the tiles (src/main.cu:261-276 builds both from one
// CSR).  It is taken only when that CSR is present and agrees with the tiles:
// A's and B's nnz equal their tiles' totals (tile_nnz[numtile], an exclusive
// scan) and every A tile row holds as many nonzeros as the CSR rows it covers.
// Otherwise the tile payloads are used (the payload route), so a caller whose
// CSR and tiles disagree IN THESE COUNTS gets C of the tiles, as from the
// reference.  Only counts are compared up front: a CSR with the same counts but
// other columns is caught when one of its products falls outside step 1's tiles
// (or C's tile totals miss its nnz), and the call then reruns on the payload
// route; one whose products all land in step 1's tiles, or with the same
// pattern but other values, gives C of the CSR.
static bool csr_matches_tiles(const tsg_smatrix *A, const tsg_smatrix *B, int tm) {
    for (const tsg_smatrix *M : {A, B}) {
        if (!M->rowpointer || !M->columnindex || !M->value || !M->tile_nnz || !M->tile_ptr) return false;
        if (M->numtile < 0 || M->tile_nnz[M->numtile] != M->nnz || M->rowpointer[M->m] != M->nnz) return false;
    }
    if (A->tilem != (A->m + tm - 1) / tm) return false;
    for (int i = 0; i < A->tilem; ++i) {
        const int r0 = std::min(A->m, i * tm), r1 = std::min(A->m, (i + 1) * tm);
        const int t0 = A->tile_ptr[i], t1 = A->tile_ptr[i + 1];
        if (t0 < 0 || t1 < t0 || t1 > A->numtile) return false;
        if (A->tile_nnz[t1] - A->tile_nnz[t0] != A->rowpointer[r1] - A->rowpointer[r0]) return false;
    }
    return true;
}

// ------------------------------------------------------------------ C ABI
extern "C" {

const char *tsg_version(void) { return "tsg-mi355x 0.1 (gfx950)"; }

int tsg_device_count(int *count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        n = 0;
    }
    *count = n;
    return TSG_OK;
}

const char *tsg_status_string(int st) {
    switch (st) {
        case TSG_OK: return "ok";
        case TSG_ERR_INVALID: return "invalid argument";
        case TSG_ERR_HIP: return "HIP runtime error";
        case TSG_ERR_OOM: return "out of memory";
        case TSG_ERR_OVERFLOW: return "count overflows the int32 layout";
        case TSG_ERR_NO_DEVICE: return "no HIP device";
        case TSG_ERR_UNSUPPORTED: return "unsupported tile size / shape";
        case TSG_ERR_IO: return "Matrix-Market read error";
        default: return "unknown";
    }
}

// ---- Matrix-Market reader: same CSR order as mmio_allinone
// (src/mmio_highlevel.h:593-759).  Whole-file read + hand-rolled tokenizer.
// Optional binary CSR cache (TSG_CSR_CACHE_DIR): <dir>/<name>.<bytes>.<mtime>.tsgcsr
// holds {m, n, nnz, isSymmetric} + rowpointer + columnindex + value in the exact
// mmio_allinone order, so a large .mtx (LiveJournal, mawi) is parsed once.
static std::string csr_cache_path(const char *filename) {
    const char *dir = getenv("TSG_CSR_CACHE_DIR");
    struct stat st;
    if (!dir || !*dir || stat(filename, &st) != 0) return std::string();
    const char *base = strrchr(filename, '/');
    base = base ? base + 1 : filename;
    char tag[64];
    snprintf(tag, sizeof(tag), ".%lld.%lld.tsgcsr", (long long)st.st_size, (long long)st.st_mtime);
    return std::string(dir) + "/" + base + tag;
}

static bool csr_cache_read(const std::string &path, tsg_smatrix *A) {
    FILE *f = path.empty() ? nullptr : fopen(path.c_str(), "rb");
    if (!f) return false;
    int hdr[4];
    bool ok = fread(hdr, sizeof(int), 4, f) == 4 && hdr[0] >= 0 && hdr[1] >= 0 && hdr[2] >= 0;
    if (ok) {
        A->m = hdr[0]; A->n = hdr[1]; A->nnz = hdr[2]; A->isSymmetric = hdr[3];
        A->rowpointer = (int *)malloc(((size_t)A->m + 1) * sizeof(int));
        A->columnindex = (int *)malloc((size_t)(A->nnz ? A->nnz : 1) * sizeof(int));
        A->value = (double *)malloc((size_t)(A->nnz ? A->nnz : 1) * sizeof(double));
        ok = A->rowpointer && A->columnindex && A->value &&
             fread(A->rowpointer, sizeof(int), (size_t)A->m + 1, f) == (size_t)A->m + 1 &&
             fread(A->columnindex, sizeof(int), (size_t)A->nnz, f) == (size_t)A->nnz &&
             fread(A->value, sizeof(double), (size_t)A->nnz, f) == (size_t)A->nnz;
        if (!ok) {
            free(A->rowpointer); free(A->columnindex); free(A->value);
            memset(A, 0, sizeof(*A));
        }
    }
    fclose(f);
    return ok;
}

static void csr_cache_write(const std::string &path, const tsg_smatrix *A) {
    if (path.empty()) return;
    const std::string tmp = path + ".part";
    FILE *f = fopen(tmp.c_str(), "wb");
    if (!f) return;
    const int hdr[4] = {A->m, A->n, A->nnz, A->isSymmetric};
    bool ok = fwrite(hdr, sizeof(int), 4, f) == 4 &&
              fwrite(A->rowpointer, sizeof(int), (size_t)A->m + 1, f) == (size_t)A->m + 1 &&
              fwrite(A->columnindex, sizeof(int), (size_t)A->nnz, f) == (size_t)A->nnz &&
              fwrite(A->value, sizeof(double), (size_t)A->nnz, f) == (size_t)A->nnz;
    ok = (fclose(f) == 0) && ok;
    if (ok) rename(tmp.c_str(), path.c_str());
    else remove(tmp.c_str());
}

static int mmio_parse(const char *filename, tsg_smatrix *A);

int tsg_mmio_allinone(const char *filename, tsg_smatrix *A) {
    if (!filename || !A) return TSG_ERR_INVALID;
    memset(A, 0, sizeof(*A));
    const std::string cache = csr_cache_path(filename);
    if (csr_cache_read(cache, A)) return TSG_OK;
    const int rc = mmio_parse(filename, A);
    if (rc == TSG_OK) csr_cache_write(cache, A);
    return rc;
}

static int mmio_parse(const char *filename, tsg_smatrix *A) {
    FILE *f = fopen(filename, "rb");
    if (!f) return TSG_ERR_IO;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<char> buf((size_t)sz + 1);
    if (sz > 0 && fread(buf.data(), 1, (size_t)sz, f) != (size_t)sz) {
        fclose(f);
        return TSG_ERR_IO;
    }
    fclose(f);
    buf[sz] = 0;
    char *p = buf.data(), *end = buf.data() + sz;
    // banner
    char *eol = (char *)memchr(p, '\n', end - p);
    if (!eol) eol = end;
    std::string banner(p, eol);
    for (auto &ch : banner) ch = (char)tolower(ch);
    char t0[64] = {0}, t1[64] = {0}, t2[64] = {0}, t3[64] = {0}, t4[64] = {0};
    if (sscanf(banner.c_str(), "%63s %63s %63s %63s %63s", t0, t1, t2, t3, t4) != 5) return TSG_ERR_IO;
    if (strncmp(t0, "%%matrixmarket", 14) != 0 || strcmp(t1, "matrix") != 0) return TSG_ERR_IO;
    if (strcmp(t2, "coordinate") != 0) return TSG_ERR_UNSUPPORTED;
    const bool is_real = !strcmp(t3, "real"), is_cplx = !strcmp(t3, "complex");
    const bool is_int = !strcmp(t3, "integer"), is_pat = !strcmp(t3, "pattern");
    if (!(is_real || is_cplx || is_int || is_pat)) return TSG_ERR_UNSUPPORTED;
    const bool sym = !strcmp(t4, "symmetric") || !strcmp(t4, "hermitian");
    p = (eol < end) ? eol + 1 : end;
    while (p < end && *p == '%') {  // comment lines
        char *q = (char *)memchr(p, '\n', end - p);
        p = q ? q + 1 : end;
    }
    char *q;
    long m = strtol(p, &q, 10); p = q;
    long n = strtol(p, &q, 10); p = q;
    long nz = strtol(p, &q, 10); p = q;
    if (m < 0 || n < 0 || nz < 0 || m > 0x7fffffff || n > 0x7fffffff) return TSG_ERR_IO;
    // Entry lines are parsed in parallel chunks cut at line starts (file order is
    // kept: chunk c's entries follow chunk c-1's), then counted and placed serially.
    std::vector<int> ri((size_t)nz), ci((size_t)nz);
    std::vector<double> vv((size_t)nz);
    std::vector<long long> cnt((size_t)m + 1, 0);
    const size_t body = (size_t)(end - p);
    int nth = (int)std::min<size_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
    nth = (int)std::max<size_t>(1, std::min<size_t>((size_t)nth, body / (1u << 22)));  // >= 4 MiB per chunk
    std::vector<char *> cut(nth + 1);
    cut[0] = p;
    cut[nth] = end;
    for (int c = 1; c < nth; ++c) {
        char *x = p + body * c / nth;
        if (x < cut[c - 1]) x = cut[c - 1];
        char *nl = (char *)memchr(x, '\n', end - x);
        cut[c] = nl ? nl + 1 : end;
    }
    struct Part {
        std::vector<int> i, j;
        std::vector<double> x;
        bool bad = false;
    };
    std::vector<Part> parts(nth);
    auto parse = [&](int c) {
        Part &P = parts[c];
        char *a = cut[c], *e = cut[c + 1], *z;
        while (true) {
            while (a < e && isspace((unsigned char)*a)) ++a;
            if (a >= e) break;
            long i = strtol(a, &z, 10);
            if (z == a) { P.bad = true; return; }
            a = z;
            long j = strtol(a, &z, 10);
            if (z == a) { P.bad = true; return; }
            a = z;
            double x = 1.0;
            if (is_real || is_cplx) {
                x = strtod(a, &z); a = z;
                if (is_cplx) { (void)strtod(a, &z); a = z; }
            } else if (is_int) {
                x = (double)strtol(a, &z, 10); a = z;
            }
            if (i < 1 || j < 1 || i > m || j > n) { P.bad = true; return; }
            P.i.push_back((int)(i - 1));
            P.j.push_back((int)(j - 1));
            P.x.push_back(x);
        }
    };
    {
        std::vector<std::thread> th;
        for (int c = 1; c < nth; ++c) th.emplace_back(parse, c);
        parse(0);
        for (auto &t : th) t.join();
    }
    long k = 0;
    for (int c = 0; c < nth; ++c) {
        const Part &P = parts[c];
        if (P.bad || k + (long)P.i.size() > nz) return TSG_ERR_IO;
        std::copy(P.i.begin(), P.i.end(), ri.begin() + k);
        std::copy(P.j.begin(), P.j.end(), ci.begin() + k);
        std::copy(P.x.begin(), P.x.end(), vv.begin() + k);
        k += (long)P.i.size();
    }
    if (k != nz) return TSG_ERR_IO;
    for (long e = 0; e < nz; ++e) cnt[ri[e]]++;
    if (sym)
        for (long k = 0; k < nz; ++k)
            if (ri[k] != ci[k]) cnt[ci[k]]++;
    long long run = 0;
    for (long r = 0; r <= m; ++r) {
        long long v = cnt[r];
        cnt[r] = run;
        run += v;
    }
    if (run > 0x7fffffffLL) return TSG_ERR_OVERFLOW;
    A->m = (int)m; A->n = (int)n; A->nnz = (int)run; A->isSymmetric = sym ? 1 : 0;
    A->rowpointer = (int *)malloc(((size_t)m + 1) * sizeof(int));
    A->columnindex = (int *)malloc((size_t)(run ? run : 1) * sizeof(int));
    A->value = (double *)malloc((size_t)(run ? run : 1) * sizeof(double));
    if (!A->rowpointer || !A->columnindex || !A->value) return TSG_ERR_OOM;
    for (long r = 0; r <= m; ++r) A->rowpointer[r] = (int)cnt[r];
    std::vector<int> fill((size_t)m + 1, 0);
    for (long k = 0; k < nz; ++k) {
        int r = ri[k], c = ci[k];
        int d = A->rowpointer[r] + fill[r]++;
        A->columnindex[d] = c;
        A->value[d] = vv[k];
        if (sym && r != c) {
            d = A->rowpointer[c] + fill[c]++;
            A->columnindex[d] = r;
            A->value[d] = vv[k];
        }
    }
    return TSG_OK;
}

void tsg_values_pos_mod10(tsg_smatrix *A) {
    for (int k = 0; k < A->nnz; ++k) A->value[k] = (double)(k % 10);
}

void tsg_matrix_destroy(tsg_smatrix *M) {
    if (!M) return;
    free(M->value); free(M->columnindex); free(M->rowpointer);
    free_tile_fields(M);
    memset(M, 0, sizeof(*M));
}

int tsg_transpose(const tsg_smatrix *A, tsg_smatrix *B) {
    if (!A || !B) return TSG_ERR_INVALID;
    HostLease lease;
    TSG_TRY(lease.acquire());
    Context &cx = lease.cx();
    hipStream_t s = lease.stream();
    tsg_dev_csr dA, dB;
    TSG_TRY(upload_csr(cx, A, dA, s));
    TSG_TRY(dev_transpose(cx, dA, dB, s));
    memset(B, 0, sizeof(*B));
    B->m = dB.m; B->n = dB.n; B->nnz = dB.nnz;
    TSG_TRY(download(&B->rowpointer, dB.rowpointer, (size_t)dB.m + 1, s));
    TSG_TRY(download(&B->columnindex, dB.columnindex, (size_t)dB.nnz, s));
    TSG_TRY(download(&B->value, dB.value, (size_t)dB.nnz, s));
    TSG_HIP(hipStreamSynchronize(s));
    cx.pool.release_all_live();
    return TSG_OK;
}

int tsg_nnzcub(const tsg_smatrix *A, const tsg_smatrix *B, unsigned long long *out) {
    if (!A || !B || !out || A->n != B->m) return TSG_ERR_INVALID;
    HostLease lease;
    TSG_TRY(lease.acquire());
    Context &cx = lease.cx();
    hipStream_t s = lease.stream();
    tsg_dev_csr dA, dB;
    TSG_TRY(upload_csr(cx, A, dA, s));
    TSG_TRY(upload(cx, &dB.rowpointer, B->rowpointer, (size_t)B->m + 1, s));
    unsigned long long *d = nullptr;
    TSG_TRY(cx.get(&d, 1));
    TSG_TRY(launch_nnzcub(cx, dA, dB, d, s));
    TSG_HIP(hipMemcpyAsync(out, d, sizeof(*out), hipMemcpyDeviceToHost, s));
    TSG_HIP(hipStreamSynchronize(s));
    cx.pool.release_all_live();
    return TSG_OK;
}

int tsg_csr2tile_row_major(tsg_smatrix *A, int tm, int tn) {
    if (!A || !valid_tiles(tm, tn)) return TSG_ERR_INVALID;
    if (!tile_side_supported(tm) || !tile_side_supported(tn)) return TSG_ERR_UNSUPPORTED;
    HostLease lease;
    TSG_TRY(lease.acquire());
    Context &cx = lease.cx();
    hipStream_t s = lease.stream();
    tsg_dev_csr d;
    tsg_dev_tiles t;
    TSG_TRY(upload_csr(cx, A, d, s));
    int rc = dev_csr2tile_row_major(cx, d, tm, tn, t, s);
    if (rc == TSG_OK) rc = download_tiles(t, A, false, s);
    cx.pool.release_all_live();
    return rc;
}

int tsg_csr2tile_col_major(tsg_smatrix *B, int tm, int tn) {
    if (!B || !valid_tiles(tm, tn)) return TSG_ERR_INVALID;
    if (!tile_side_supported(tm) || !tile_side_supported(tn)) return TSG_ERR_UNSUPPORTED;
    HostLease lease;
    TSG_TRY(lease.acquire());
    Context &cx = lease.cx();
    hipStream_t s = lease.stream();
    tsg_dev_csr d;
    tsg_dev_tiles t;
    TSG_TRY(upload_csr(cx, B, d, s));
    int rc = dev_csr2tile_col_major(cx, d, tm, tn, t, s);
    if (rc == TSG_OK) rc = download_tiles(t, B, true, s);
    cx.pool.release_all_live();
    return rc;
}

int tsg_tilespgemm(tsg_smatrix *A, tsg_smatrix *B, tsg_smatrix *C, unsigned int *bmA, unsigned int *bmB,
                   int bmlen, double densityA, double densityB, unsigned long long nnzCub,
                   unsigned long long *nnzC_computed, double *compression_rate, double *time_tile,
                   double *gflops_tile, const char *filename, double *time_step1, double *time_step2,
                   double *time_step3, double *time_malloc, int tm, int tn) {
    (void)bmA; (void)bmB; (void)bmlen; (void)densityA; (void)densityB; (void)filename;
    if (!A || !B || !C || !valid_tiles(tm, tn)) return TSG_ERR_INVALID;
    if (!tile_side_supported(tm) || !tile_side_supported(tn)) return TSG_ERR_UNSUPPORTED;
    if (A->n != B->m || !A->tile_ptr || !B->tile_ptr || !B->mask || !B->csc_tile_ptr) return TSG_ERR_INVALID;
    // 16x16: the staged pipeline's tile-payload kernels; other sizes (32/48/64 x
    // 16/32/48/64): step 1 at that size plus the general-size step-2/3 kernels
    // (tsg_tile_steps.hip) -- steps 1-3 all run natively at tm x tn
    const bool sq16 = tile_size_supported(tm, tn);
    HostLease lease;
    TSG_TRY(lease.acquire());
    Context &cx = lease.cx();
    hipStream_t s = lease.stream();
    tsg_dev_tiles dA, dB, dC;
    // The reference's SMatrix carries the CSR beside the tiles (src/main.cu builds
    // both).  When both operands have it and B's rows are column-sorted, C comes
    // from the device CSR route and the tiled layout kernel (below): then only
    // the tile STRUCTURES of A and B are read (step 1), and only they are copied
    // in -- no tile payloads, no B row-major views.  Copies are outside the timed
    // region, as in the reference.  TSG_TILED_CSR=0 keeps the tile-payload kernels.
    tsg_dev_csr cA{}, cB{};
    bool use_csr = false, bsorted = false;
    {
        const char *e = getenv("TSG_TILED_CSR");
        const bool allow = !(e && !strcmp(e, "0"));
        if (sq16 && allow && csr_matches_tiles(A, B, tm)) {
            TSG_TRY(upload_csr(cx, A, cA, s));
            TSG_TRY(upload_csr(cx, B, cB, s));
            use_csr = true;  // (if B's rows turn out column-sorted: checked inside the timed region)
        }
    }
    if (use_csr) {
        TSG_TRY(upload_tile_structure(cx, A, tm, tn, dA, s));
        TSG_TRY(upload_tile_structure(cx, B, tn, tm, dB, s));
    } else {
        TSG_TRY(upload_tiles(cx, A, tm, tn, false, dA, s));
        TSG_TRY(upload_tiles(cx, B, tn, tm, true, dB, s));
    }
    TSG_HIP(hipStreamSynchronize(s));
    tsg_stats st{};
    auto h0 = std::chrono::steady_clock::now();
    if (use_csr) {
        // B's sortedness decides the route: work of the call, so inside the timed
        // region.  Unsorted rows (rare) take the tile payloads after all, whose
        // copies then fall inside it too (the pool keeps the structures until
        // the call's end).
        TSG_TRY(dev_rows_sorted(cx, cB, &bsorted, s));
        use_csr = bsorted;
        if (!use_csr) {
            TSG_TRY(upload_tiles(cx, A, tm, tn, false, dA, s));
            TSG_TRY(upload_tiles(cx, B, tn, tm, true, dB, s));
            TSG_HIP(hipStreamSynchronize(s));
        }
    }
    int rc;
    int evi[4] = {0, 1, 2, 3};  // the events bracketing steps 1 | 2 | 3
    HostLease aux;  // the CSR route's step 1: its own context and stream (outlives the download)
    double t_s1 = -1.0;
    if (sq16 && use_csr) {
        // step 1: the reference's tile-pattern C structure (empty tiles included);
        // steps 2 + 3: C's nonzeros on the device CSR route (banded / row-merge /
        // staged) -- bit-identical to the reference's steps 2/3 +
        // tile2csr -- then laid out as the reference's tiled C on step 1's
        // structure (tsg_ctiles.hip): Ptr, masks, Col, Value, tile_nnz.
        // Step 1 and the CSR product read only A and B: step 1 runs on a second
        // stream from a host thread (each has host round trips of its own), the
        // layout kernel joins them.
        evi[0] = 12, evi[1] = 12, evi[2] = 13, evi[3] = 14;
        dC = tsg_dev_tiles{};
        dC.m = A->m; dC.n = B->n; dC.tile_m = 16; dC.tile_n = 16;
        dC.tilem = dA.tilem; dC.tilen = dB.tilen;
        TSG_TRY(aux.acquire());
        Context &cx1 = aux.cx();
        hipStream_t s1 = aux.stream();
        int rc1 = TSG_OK;
        // (the step times' markers only with TSG_STAGE_EVENTS=1: each cost a few
        // us of GPU time on a ~1 ms call; the steps report 0 without them)
        const char *sev = getenv("TSG_STAGE_EVENTS");
        const bool se = sev && sev[0] == '1';
        auto step1 = [&] {
            long long tp = 0;
            rc1 = hipSetDevice(cx.device) == hipSuccess ? TSG_OK : TSG_ERR_HIP;
            if (rc1 == TSG_OK && se) rc1 = hipEventRecord(cx1.ev[11], s1) == hipSuccess ? TSG_OK : TSG_ERR_HIP;
            if (rc1 == TSG_OK) rc1 = dev_step1(cx1, dA, dB, dC, &tp, s1);
            if (rc1 == TSG_OK && se) rc1 = hipEventRecord(cx1.ev[12], s1) == hipSuccess ? TSG_OK : TSG_ERR_HIP;
            if (rc1 == TSG_OK) rc1 = hipStreamSynchronize(s1) == hipSuccess ? TSG_OK : TSG_ERR_HIP;
        };
        // step 1 from a host thread of its own; when the thread cannot be made
        // (std::system_error: no exception may leave this C ABI) it runs here,
        // before the product, on its own stream
        std::thread th;
        bool threaded = true;
        try {
            th = std::thread(step1);
        } catch (...) {
            threaded = false;
            step1();
        }
        tsg_dev_csr Cc{};
        rc = se && hipEventRecord(cx.ev[12], s) != hipSuccess ? TSG_ERR_HIP : TSG_OK;
        if (rc == TSG_OK) rc = dev_spgemm16(cx, &cA, &cB, s, &Cc, nullptr, bsorted ? 1 : -1);
        if (rc == TSG_OK && se) rc = hipEventRecord(cx.ev[13], s) == hipSuccess ? TSG_OK : TSG_ERR_HIP;
        if (threaded) th.join();
        if (rc == TSG_OK) rc = rc1;
        if (rc == TSG_OK) t_s1 = se ? ev_ms(cx1.ev[11], cx1.ev[12]) : 0.0;
        if (rc == TSG_OK) rc = dev_ctiles_from_csr(cx, Cc, dC, s);
        if (rc == TSG_OK && se) rc = hipEventRecord(cx.ev[14], s) == hipSuccess ? TSG_OK : TSG_ERR_HIP;
        if (!se) evi[0] = evi[1] = evi[2] = evi[3] = -1;  // (no step times)
        if (rc == TSG_OK) TSG_HIP(hipStreamSynchronize(s));
        // a nonzero of the CSR product outside step 1's tiles, or tile totals that
        // miss nnz(C): the CSR disagrees with the tiles it was passed with (same
        // counts, other columns) -- C of the tile payloads after all, as from the
        // reference, the payloads' copies inside the timed region (this call's work)
        if (rc == TSG_OK && cx.pinned[8] != 0) {
            use_csr = false;
            evi[0] = 0, evi[1] = 1, evi[2] = 2, evi[3] = 3;
            t_s1 = -1.0;
            rc = upload_tiles(cx, A, tm, tn, false, dA, s);
            if (rc == TSG_OK) rc = upload_tiles(cx, B, tn, tm, true, dB, s);
            dC = tsg_dev_tiles{};
            if (rc == TSG_OK) rc = dev_tilespgemm(cx, dA, dB, dC, &st, s, cx.ev, nullptr, nullptr, nullptr, false);
        }
    } else if (sq16) {
        rc = dev_tilespgemm(cx, dA, dB, dC, &st, s, cx.ev, nullptr, nullptr, nullptr, false);
    } else {
        dC = tsg_dev_tiles{};
        dC.m = A->m; dC.n = B->n; dC.tile_m = tm; dC.tile_n = tm;
        dC.tilem = dA.tilem; dC.tilen = dB.tilen;
        long long tp = 0;
        rc = hipEventRecord(cx.ev[0], s) == hipSuccess ? TSG_OK : TSG_ERR_HIP;
        if (rc == TSG_OK) rc = dev_step1(cx, dA, dB, dC, &tp, s);
        if (rc == TSG_OK) rc = dev_tile_steps23(cx, dA, dB, dC, s, cx.ev);
    }
    if (rc == TSG_OK) TSG_HIP(hipStreamSynchronize(s));
    auto h1 = std::chrono::steady_clock::now();
    // (the CSR route's layout kernel already wrote the empty tiles' Ptr and mask)
    if (rc == TSG_OK) rc = dev_tiles_finalize_c(cx, dC, s, !(sq16 && use_csr));
    if (rc == TSG_OK) {
        memset(C, 0, sizeof(*C));
        C->m = dC.m; C->n = dC.n; C->nnz = dC.nnz;
        rc = download_tiles(dC, C, false, s);
    }
    cx.pool.release_all_live();
    if (rc != TSG_OK) return rc;
    // the reference's steps at every tile size: step 1 | step 2 + scan | step 3
    // (the CSR route: step 1 overlaps step 2, its own stream's duration)
    const bool stepev = evi[0] >= 0;
    const double t1 = t_s1 >= 0 ? t_s1 : (stepev ? ev_ms(cx.ev[evi[0]], cx.ev[evi[1]]) : 0.0),
                 t2 = stepev ? ev_ms(cx.ev[evi[1]], cx.ev[evi[2]]) : 0.0,
                 t3 = stepev ? ev_ms(cx.ev[evi[2]], cx.ev[evi[3]]) : 0.0;
    const double tk = std::chrono::duration<double, std::milli>(h1 - h0).count();
    if (time_step1) *time_step1 = t1;
    if (time_step2) *time_step2 = t2;
    if (time_step3) *time_step3 = t3;
    if (time_malloc) *time_malloc = tk - (t1 + t2 + t3) > 0 ? tk - (t1 + t2 + t3) : 0.0;
    if (time_tile) *time_tile = tk;
    if (nnzC_computed) *nnzC_computed = (unsigned long long)C->nnz;
    if (compression_rate) *compression_rate = C->nnz ? (double)nnzCub / (double)C->nnz : 0.0;
    if (gflops_tile) *gflops_tile = tk > 0 ? 2.0 * (double)nnzCub / (tk * 1e6) : 0.0;
    if (!quiet()) {
        printf("step1 ---------------------- Runtime is  %.2f ms-------------------------\n", t1);
        printf("step2 ---------------------- Runtime is  %.2f ms-------------------------\n", t2);
        printf("step3 ---------------------- Runtime is  %.2f ms------------------------\n", t3);
        printf("Non-empty tiles of C = %i\n", C->numtile);
        printf("nnzC = %i\n", C->nnz);
        printf("CUDA  TileSpGEMM runtime is %4.2f ms, gflops = %4.2f\n", tk,
               tk > 0 ? 2.0 * (double)nnzCub / (tk * 1e6) : 0.0);
    }
    return TSG_OK;
}

int tsg_tile2csr(tsg_smatrix *C, int tm, int tn) {
    (void)tn;
    if (!C || !C->tile_ptr || !valid_tiles(tm, tm)) return TSG_ERR_INVALID;
    if (!tile_side_supported(tm)) return TSG_ERR_UNSUPPORTED;
    HostLease lease;
    TSG_TRY(lease.acquire());
    Context &cx = lease.cx();
    hipStream_t s = lease.stream();
    tsg_dev_tiles t;
    tsg_dev_csr d;
    TSG_TRY(upload_tiles(cx, C, tm, tm, false, t, s));
    int rc = dev_tile2csr(cx, t, d, s);
    if (rc == TSG_OK) {
        free(C->rowpointer); free(C->columnindex); free(C->value);
        rc = download(&C->rowpointer, d.rowpointer, (size_t)C->m + 1, s);
        if (rc == TSG_OK) rc = download(&C->columnindex, d.columnindex, (size_t)d.nnz, s);
        if (rc == TSG_OK) rc = download(&C->value, d.value, (size_t)d.nnz, s);
        if (rc == TSG_OK && hipStreamSynchronize(s) != hipSuccess) rc = TSG_ERR_HIP;
        C->nnz = d.nnz;
    }
    cx.pool.release_all_live();
    return rc;
}

// ---- device-resident API
int tsg_context_create(int device, tsg_context **ctx) {
    if (!ctx) return TSG_ERR_INVALID;
    TSG_TRY(check_device());
    tsg_context *c = new tsg_context();
    int rc = c->cx.init(device);
    if (rc != TSG_OK) {
        delete c;
        return rc;
    }
    *ctx = c;
    return TSG_OK;
}

int tsg_context_destroy(tsg_context *ctx) {
    if (!ctx) return TSG_ERR_INVALID;
    ctx->cx.destroy();
    delete ctx;
    return TSG_OK;
}

int tsg_context_reset(tsg_context *ctx) {
    if (!ctx) return TSG_ERR_INVALID;
    ctx->cx.pool.release_all_live();
    return TSG_OK;
}

int tsg_dev_malloc(tsg_context *ctx, void **ptr, size_t bytes) {
    if (!ctx || !ptr) return TSG_ERR_INVALID;
    return ctx->cx.pool.alloc(ptr, bytes);
}

int tsg_dev_free(tsg_context *ctx, void *ptr) {
    if (!ctx) return TSG_ERR_INVALID;
    ctx->cx.pool.release(ptr);
    return TSG_OK;
}

int tsg_memcpy_h2d(tsg_context *ctx, void *dst, const void *src, size_t bytes, void *stream) {
    (void)ctx;
    TSG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    TSG_HIP(hipStreamSynchronize((hipStream_t)stream));
    return TSG_OK;
}

int tsg_memcpy_d2h(tsg_context *ctx, void *dst, const void *src, size_t bytes, void *stream) {
    (void)ctx;
    TSG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    TSG_HIP(hipStreamSynchronize((hipStream_t)stream));
    return TSG_OK;
}

int tsg_memcpy_d2d(tsg_context *ctx, void *dst, const void *src, size_t bytes, void *stream) {
    (void)ctx;
    TSG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    TSG_HIP(hipStreamSynchronize((hipStream_t)stream));
    return TSG_OK;
}

int tsg_dev_csr2tile_row_major(tsg_context *ctx, const tsg_dev_csr *A, int tm, int tn, void *stream,
                               tsg_dev_tiles *out) {
    if (!ctx || !A || !out || !valid_tiles(tm, tn)) return TSG_ERR_INVALID;
    return dev_csr2tile_row_major(ctx->cx, *A, tm, tn, *out, (hipStream_t)stream);
}

int tsg_dev_csr2tile_col_major(tsg_context *ctx, const tsg_dev_csr *B, int tm, int tn, void *stream,
                               tsg_dev_tiles *out) {
    if (!ctx || !B || !out || !valid_tiles(tm, tn)) return TSG_ERR_INVALID;
    return dev_csr2tile_col_major(ctx->cx, *B, tm, tn, *out, (hipStream_t)stream);
}

int tsg_dev_tilespgemm(tsg_context *ctx, const tsg_dev_tiles *A, const tsg_dev_tiles *B, void *stream,
                       tsg_dev_tiles *C, tsg_stats *stats) {
    if (!ctx || !A || !B || !C) return TSG_ERR_INVALID;
    if (!B->tile_rm2csc || !B->rm_mask || !B->rm_rowstart) return TSG_ERR_INVALID;
    return dev_tilespgemm(ctx->cx, *A, *B, *C, stats, (hipStream_t)stream, nullptr, nullptr);
}

int tsg_dev_tile2csr(tsg_context *ctx, const tsg_dev_tiles *C, void *stream, tsg_dev_csr *out) {
    if (!ctx || !C || !out) return TSG_ERR_INVALID;
    return dev_tile2csr(ctx->cx, *C, *out, (hipStream_t)stream);
}

int tsg_dev_transpose(tsg_context *ctx, const tsg_dev_csr *A, void *stream, tsg_dev_csr *out) {
    if (!ctx || !A || !out) return TSG_ERR_INVALID;
    return dev_transpose(ctx->cx, *A, *out, (hipStream_t)stream);
}

static void release_tiles(Context &cx, tsg_dev_tiles &t) {
    void *ps[] = {t.tile_ptr, t.tile_columnidx, t.tile_rowidx, t.tile_nnz, t.tile_csr_Ptr,
                  t.tile_csr_Col, t.tile_csr_Value, t.mask, t.csc_tile_ptr, t.csc_tile_rowidx,
                  t.tile_rm2csc, t.rm_mask, t.rm_rowstart};
    for (void *p : ps) cx.put(p);
    t = tsg_dev_tiles{};
}


// CSR in -> CSR out through the 16x16 tiled pipeline (C does not depend on the
// tile size; other sizes are a layout choice of the host tile API).
static int dev_spgemm16(Context &cx, const tsg_dev_csr *A, const tsg_dev_csr *B, hipStream_t s, tsg_dev_csr *C,
                        tsg_stats *stats, int b_sorted) {
    const int tm = 16, tn = 16;
    tsg_stats st{};
    tsg_dev_tiles tA, tB, tC;
    auto h0 = std::chrono::steady_clock::now();
    // the stage events (ev 8, 9, 0, 1, 3) only on request: each marker on the
    // stream cost ~2-3 us of GPU time (cant 0.707 -> 0.692 ms without them, r5e1);
    // the kernel bracket (ev 4, 5) and the end (ev 10) always
    {
        const char *se = getenv("TSG_STAGE_EVENTS");
        cx.stage_ev = se && se[0] == '1';
    }
    // (no stats asked for -- the tiled route's product, a caller passing NULL:
    // not even the numeric phase's bracket on the row-merge and banded paths)
    hipEvent_t *const evp = stats || cx.stage_ev ? cx.ev : nullptr;
    if (cx.stage_ev) TSG_HIP(hipEventRecord(cx.ev[8], s));
    // Element streaming (steps 2/3 straight from the CSR operands) needs B's rows
    // column-sorted.  Sparse tiles (few nonzeros per A tile, e.g. web graphs) then
    // need only the tile STRUCTURE of A and B; denser tiles keep the full
    // csr2tile payloads for step 2's tile-level mask ORs.
    // The sortedness check is queued ahead of A's tile counts; both results come
    // back with the counts' host round trip.  (With unsorted B rows the counts are
    // discarded: the full csr2tile below rebuilds A's tiles.)
    // (its last step -- the shares' sum into the flag -- rides on the row-merge
    // setup's binning kernel, or runs before the first read-back of another route)
    SortedShares shares;
    // (A referencing at most 1/64 of B's rows -- the mawi prefix: 6,828 entries
    // against 226 M rows -- only the B rows A references are checked, 0.88 ->
    // 0.12 ms there; a LiveJournal hub block's 125 K entries reach hub rows
    // whose entries outweigh the whole-B sweep: 0.19 vs 0.10 ms, so it keeps
    // the sweep.  The staged tile pipeline, which reads whole B tile rows,
    // re-checks all of B below.)
    const bool ref_check = b_sorted != 1 && (long long)A->nnz * 64 < (long long)B->m;
    if (b_sorted == 1)
        cx.pinned[1] = 0;  // (known: no check, no shares for the binning kernel to sum)
    else if (ref_check)
        TSG_TRY(dev_rows_sorted_shares_ref(cx, *A, *B, cx.pinned + 1, &shares, s));
    else
        TSG_TRY(dev_rows_sorted_shares(cx, *B, cx.pinned + 1, &shares, s));
    // Routing, B's rows column-sorted:
    //  * banded path (tsg_band.hip) when A averages >= 8 entries per row and every
    //    C row's reachable columns fit one window of <= 2,048 columns holding at
    //    least as many products as columns (FEM-like: cant); its check is a
    //    statistics kernel + one host round trip;
    //  * otherwise the row-merge setup (entry table, classes) + one round trip:
    //    the row-merge path (tsg_rows.hip) for every product whose B rows are
    //    strictly column-sorted, hub rows included (dominant-run / windowed
    //    kernels), unless a row holds more than 2^31 - 1 products
    //    (dev_rows_accept);
    //  * the staged tile pipeline below for the rest and for unsorted B rows
    //    (or rows repeating a column).
    // TSG_PATH=band / rows / tiles forces a path (band when its check passes).
    const char *path = getenv("TSG_PATH");
    const bool force_tiles = path && !strcmp(path, "tiles");
    const bool force_band = path && !strcmp(path, "band"), force_rows = path && !strcmp(path, "rows");
    if (!force_tiles) {
        bool band = false;
        BandWin bw;
        // band candidates first (A rows of >= 8 entries on average): the window
        // check's read-back also brings the sortedness flag
        if (!force_rows && (force_band || (A->m > 0 && A->nnz >= 8LL * A->m))) {
            TSG_TRY(dev_band_check(cx, *A, *B, force_band, &band, &bw, s, &shares));  // (sums the shares too)
        }
        if (band && cx.pinned[1] != 0) {  // unsorted B rows: the windows mean nothing
            cx.put(bw.win);
            cx.put(bw.width);
            cx.put(bw.ebnd);
            band = false;
        }
        long long path_id = -1;
        if (cx.stage_ev) TSG_HIP(hipEventRecord(cx.ev[9], s));
        if (band) {
            const int rc = dev_spgemm_band(cx, *A, *B, bw, *C, &st, s, evp);
            cx.put(bw.win);
            cx.put(bw.width);
            cx.put(bw.ebnd);
            TSG_TRY(rc);
            path_id = TSG_PATH_BAND;
        } else {
            // the row-merge setup and the sortedness flag: one host round trip
            // decides rows / tiles
            if (cx.stage_ev) TSG_HIP(hipEventRecord(cx.ev[0], s));
            RowsPlan plan;
            TSG_TRY(dev_rows_setup_async(cx, *A, *B, plan, s, shares.part ? &shares : nullptr));
            TSG_TRY(stream_wait(s));
            dev_rows_setup_read(cx, plan);
            const bool bsorted0 = cx.pinned[1] == 0;
            if (bsorted0 && !force_band && (force_rows || dev_rows_accept(plan))) {
                TSG_TRY(dev_rows_run(cx, *A, *B, plan, *C, &st, s, evp));
                path_id = TSG_PATH_ROWS;
            } else {
                dev_rows_release(cx, plan);
            }
        }
        if (path_id >= 0) {
            if (!evp) {  // (C complete on return, no marker)
                TSG_TRY(stream_wait(s));
                return TSG_OK;
            }
            // (the path returned with its stream drained; the end marker only for
            // the stage times -- its record and synchronisation cost a few us a call)
            if (cx.stage_ev) TSG_HIP(hipEventRecord(cx.ev[10], s));
            TSG_TRY(stream_wait(s));
            auto h1 = std::chrono::steady_clock::now();
            st.numtileA = -1;
            st.numtileB = -1;
            st.path = path_id;
            // (stage times 0 without the stage events: unmeasured, not free)
            const bool se = cx.stage_ev;
            st.t_csr2tile_ms = se ? ev_ms(cx.ev[8], cx.ev[9]) : 0.0;  // sortedness (+ band: window statistics)
            st.t_step1_ms = se ? ev_ms(cx.ev[0], cx.ev[1]) : 0.0;     // entry table, classes / row windows / units
            st.t_step2_ms = 0.0;                                      // (structure and values together)
            st.t_step3_ms = se ? ev_ms(cx.ev[1], cx.ev[3]) : 0.0;     // the row / unit kernels, scan, compaction
            st.t_step3_kernel_ms = ev_ms(cx.ev[4], cx.ev[5]);
            st.t_tile2csr_ms = 0.0;                                   // (fused)
            st.t_kern_ms = se ? ev_ms(cx.ev[0], cx.ev[3]) : 0.0;
            st.t_e2e_ms = std::chrono::duration<double, std::milli>(h1 - h0).count();
            st.t_malloc_ms = se ? st.t_e2e_ms - ev_ms(cx.ev[8], cx.ev[10]) : 0.0;
            if (st.t_malloc_ms < 0) st.t_malloc_ms = 0;
            if (stats) *stats = st;
            return TSG_OK;
        }
    }
    TSG_TRY(dev_rows_sorted_finish(cx, shares, s));  // (forced tiles: the flag is still owed)
    if (ref_check) {  // (the referenced rows' flag: the tile pipeline needs all of B's)
        bool all_sorted = false;
        TSG_TRY(dev_rows_sorted(cx, *B, &all_sorted, s));
    }
    if (!cx.stage_ev) TSG_HIP(hipEventRecord(cx.ev[8], s));  // (the staged pipeline: its stage times always)
    const char *md = getenv("TSG_STEP2_MODE");
    const int forced = !md ? -1 : !strcmp(md, "elem") ? 1 : !strcmp(md, "tile") ? 0 : -1;
    const double skip = forced == 1 ? 1e300 : forced == 0 ? 0.0 : kStep2ElemMaxTileDensity;
    TSG_TRY(dev_tile_structure(cx, *A, tm, tn, tA, s, skip));  // synchronises the stream
    const bool bsorted = cx.pinned[1] == 0;
    const bool alias = A->rowpointer == B->rowpointer && A->columnindex == B->columnindex && A->m == B->m &&
                       A->n == B->n && tm == tn;
    bool s2elem = false, b_is_a = false;
    if (bsorted) {
        // tile STRUCTURE of A and B from CSR; denser tiles add the row masks that
        // step 2's tile-level ORs read (no sort-based csr2tile on this path)
        // element streaming throughout (sparse tiles) builds C's structure from the
        // CSR operands: then A's and B's tile counts are all that is needed
        s2elem = forced >= 0 ? forced == 1 : (double)A->nnz < kStep2ElemMaxTileDensity * (double)tA.numtile;
        if (alias) {
            tB = tA;
            b_is_a = true;
        } else {
            const int rc = dev_tile_structure(cx, *B, tn, tm, tB, s, s2elem ? 1e300 : 0.0);
            if (rc == TSG_ERR_UNSUPPORTED && s2elem) {
                // B's tile count is a statistic on the element path (steps 1-3 read
                // B's CSR).  A B too wide for the (tile row, window) count units --
                // e.g. mawi, 14 M tile rows x 216 windows -- is reported as -1.
                tB = tsg_dev_tiles{};
                tB.m = B->m; tB.n = B->n; tB.nnz = B->nnz;
                tB.tile_m = tn; tB.tile_n = tm;
                tB.tilem = (B->m + tn - 1) / tn;
                tB.tilen = (B->n + tm - 1) / tm;
                tB.numtile = -1;
            } else {
                TSG_TRY(rc);
            }
        }
        if (!s2elem) {
            TSG_TRY(dev_tile_masks(cx, *A, tA, &tA.mask, s));
            if (b_is_a) tB.rm_mask = tA.mask;
            else TSG_TRY(dev_tile_masks(cx, *B, tB, &tB.rm_mask, s));
        }
    } else {  // unsorted B rows: full csr2tile, tile-payload steps 2 and 3
        release_tiles(cx, tA);
        TSG_TRY(dev_csr2tile_row_major(cx, *A, tm, tn, tA, s));
        TSG_TRY(dev_csr2tile_col_major(cx, *B, tm, tn, tB, s));
    }
    TSG_HIP(hipEventRecord(cx.ev[9], s));
    // tile2csr is fused into step 3's epilogue on this path (C tiles stay materialised)
    TSG_TRY(dev_tilespgemm(cx, tA, tB, tC, &st, s, cx.ev, C, bsorted ? A : nullptr, bsorted ? B : nullptr,
                           s2elem));
    TSG_HIP(hipEventRecord(cx.ev[10], s));
    TSG_HIP(hipEventSynchronize(cx.ev[10]));
    auto h1 = std::chrono::steady_clock::now();
    st.numtileA = tA.numtile;
    st.numtileB = tB.numtile;
    st.t_csr2tile_ms = ev_ms(cx.ev[8], cx.ev[9]);
    st.t_step1_ms = ev_ms(cx.ev[0], cx.ev[1]);
    st.t_step2_ms = ev_ms(cx.ev[1], cx.ev[2]);
    st.t_step3_ms = ev_ms(cx.ev[2], cx.ev[3]);
    st.t_step3_kernel_ms = ev_ms(cx.ev[4], cx.ev[5]);
    st.t_tile2csr_ms = ev_ms(cx.ev[3], cx.ev[10]);
    st.t_kern_ms = ev_ms(cx.ev[0], cx.ev[3]);
    st.t_e2e_ms = std::chrono::duration<double, std::milli>(h1 - h0).count();
    st.t_malloc_ms = st.t_e2e_ms - ev_ms(cx.ev[8], cx.ev[10]);
    if (st.t_malloc_ms < 0) st.t_malloc_ms = 0;
    release_tiles(cx, tA);
    if (b_is_a) tB = tsg_dev_tiles{};
    release_tiles(cx, tB);
    release_tiles(cx, tC);
    if (stats) *stats = st;
    return TSG_OK;
}

int tsg_dev_spgemm(tsg_context *ctx, const tsg_dev_csr *A, const tsg_dev_csr *B, int tm, int tn,
                   void *stream, tsg_dev_csr *C, tsg_stats *stats) {
    if (!ctx || !A || !B || !C || !valid_tiles(tm, tn) || A->n != B->m) return TSG_ERR_INVALID;
    if (!tile_side_supported(tm) || !tile_side_supported(tn)) return TSG_ERR_UNSUPPORTED;
    return dev_spgemm16(ctx->cx, A, B, (hipStream_t)stream, C, stats);
}

int tsg_dev_spgemm_sorted_b(tsg_context *ctx, const tsg_dev_csr *A, const tsg_dev_csr *B, int b_checked_sorted,
                            int tm, int tn, void *stream, tsg_dev_csr *C, tsg_stats *stats) {
    if (!ctx || !A || !B || !C || !valid_tiles(tm, tn) || A->n != B->m) return TSG_ERR_INVALID;
    if (!tile_side_supported(tm) || !tile_side_supported(tn)) return TSG_ERR_UNSUPPORTED;
    return dev_spgemm16(ctx->cx, A, B, (hipStream_t)stream, C, stats, b_checked_sorted == 1 ? 1 : -1);
}

int tsg_dev_csr_rows_sorted(tsg_context *ctx, const tsg_dev_csr *M, void *stream, int *sorted) {
    if (!ctx || !M || !sorted || M->m < 0 || M->nnz < 0) return TSG_ERR_INVALID;
    bool ok = false;
    TSG_TRY(dev_rows_sorted(ctx->cx, *M, &ok, (hipStream_t)stream));
    *sorted = ok ? 1 : 0;
    return TSG_OK;
}

int tsg_spgemm_csr(const tsg_smatrix *A, const tsg_smatrix *B, tsg_smatrix *C, int tm, int tn,
                   tsg_stats *stats) {
    if (!A || !B || !C || A->n != B->m || !valid_tiles(tm, tn)) return TSG_ERR_INVALID;
    if (!tile_side_supported(tm) || !tile_side_supported(tn)) return TSG_ERR_UNSUPPORTED;
    HostLease lease;
    TSG_TRY(lease.acquire());
    Context &cx = lease.cx();
    hipStream_t s = lease.stream();
    tsg_dev_csr dA, dB, dC;
    TSG_TRY(upload_csr(cx, A, dA, s));
    TSG_TRY(upload_csr(cx, B, dB, s));
    TSG_HIP(hipStreamSynchronize(s));
    int rc = tsg_dev_spgemm(lease.ctx(), &dA, &dB, tm, tn, s, &dC, stats);
    if (rc == TSG_OK) {
        memset(C, 0, sizeof(*C));
        C->m = dC.m; C->n = dC.n; C->nnz = dC.nnz;
        rc = download(&C->rowpointer, dC.rowpointer, (size_t)dC.m + 1, s);
        if (rc == TSG_OK) rc = download(&C->columnindex, dC.columnindex, (size_t)dC.nnz, s);
        if (rc == TSG_OK) rc = download(&C->value, dC.value, (size_t)dC.nnz, s);
        if (rc == TSG_OK && hipStreamSynchronize(s) != hipSuccess) rc = TSG_ERR_HIP;
    }
    cx.pool.release_all_live();
    return rc;
}

}  // extern "C"
