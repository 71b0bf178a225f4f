/*
 * va_reuse_probe.hip - does a virtual address mapped again to other physical
 * memory read through stale translations? (round 4: peers read old data and
 * zeros through fresh fd-based imports when the exporter's new allocation sat
 * at its old address, r04e). One process, `iters` rounds per mode; every
 * round makes a new allocation, writes the round's value into it by DMA
 * (hipMemcpy from the host) and checks it by a kernel (every word) and by DMA
 * (first and last words), then writes another value by a kernel and reads
 * that back by DMA: a stale translation on either path shows as a mismatch:
 *   same     one reservation kept; each round maps a new physical allocation
 *            at the SAME address (unmap + release between rounds)
 *   fresh    each round maps its allocation at a NEW reservation; the old
 *            one is unmapped and released but its address never freed
 *   reserve  each round reserves, maps, then unmaps, releases AND frees the
 *            address (the runtime may hand the same address out again)
 *   malloc   hipMalloc / hipFree per round
 *   same_kcopy, reserve_kcopy (round 5): same / reserve,
 *            with the upload done by a copy kernel from pinned host memory
 *            instead of the copy engine (hipMemcpy); then checked the same way
 *
 *   va_reuse_probe [iters = 200] [MiB = 6]
 *
 * Multi-process mode (round 5, VERDICT r04 next #3: round 3's data loss was
 * on hipMalloc buffers): NP processes on the one GPU, the round-3 worker
 * pattern. Every round each process hipMallocs a buffer of the same size
 * (the runtime hands out the address it freed milliseconds before), uploads
 * its (rank, round) value by DMA, checks it by a kernel, exports it
 * (hipIpcGetMemHandle), maps every peer's buffer of the round
 * (hipIpcOpenMemHandle) and checks each by a kernel and by DMA, then frees.
 *   close  imports are closed before their exporter frees
 *   hold   each import is closed a round later, after its exporter has freed
 *          it and allocated the next buffer (peers hold imports of each
 *          other's freed allocations while the address is recycled)
 *
 *   va_reuse_probe ipc <dir> <rank> <np> <iters> <MiB> <close|hold>
 *
 * Started by scripts/va_reuse_ipc.py; processes meet through files in <dir>.
 *
 * Built by `make -C tools/src` into tools/ (not part of the product).
 */
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("FAIL %s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_set(uint32_t *p, size_t n, uint32_t v)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        p[i] = v;
    }
}

__global__ void k_count(const uint32_t *p, size_t n, uint32_t v, unsigned *bad, unsigned *zero)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t x = p[i];
        if (x != v) {
            atomicAdd(bad, 1u);
            if (x == 0) atomicAdd(zero, 1u);
        }
    }
}

/* the upload as a kernel: every word read from pinned host memory (over
 * PCIe, no copy engine) */
__global__ void k_upload(uint32_t *p, const uint32_t *host, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        p[i] = host[i];
    }
}

static hipMemAllocationProp prop()
{
    hipMemAllocationProp p;
    memset(&p, 0, sizeof(p));
    p.type = hipMemAllocationTypePinned;
    p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = 0;
    return p;
}

static void map_rw(void *va, size_t bytes, hipMemGenericAllocationHandle_t h)
{
    CHECK(hipMemMap(va, bytes, 0, h, 0));
    hipMemAccessDesc d;
    memset(&d, 0, sizeof(d));
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = 0;
    d.flags = hipMemAccessFlagsProtReadWrite;
    CHECK(hipMemSetAccess(va, bytes, &d, 1));
}

struct Stats {
    int rounds = 0, kernel_bad = 0, dma_bad = 0, dma_after_kernel_bad = 0, same_va = 0;
    unsigned long long bad_words = 0, zero_words = 0;
};

static void check_round(uint32_t *p, size_t n, uint32_t v, unsigned *ctr, Stats &s,
                        bool kcopy = false)
{
    static std::vector<uint32_t> host;
    static uint32_t *pinned = nullptr;
    static size_t pinned_n = 0;
    if (kcopy) {
        if (pinned_n < n) {
            if (pinned) CHECK(hipHostFree(pinned));
            CHECK(hipHostMalloc((void**)&pinned, n * 4, hipHostMallocDefault));
            pinned_n = n;
        }
        for (size_t i = 0; i < n; i++) pinned[i] = v;
        hipLaunchKernelGGL(k_upload, dim3(1024), dim3(256), 0, 0, p, pinned, n);  /* kernel write */
        CHECK(hipDeviceSynchronize());
    } else {
        host.assign(n, v);
        CHECK(hipMemcpy(p, host.data(), n * 4, hipMemcpyHostToDevice));   /* DMA write */
    }
    CHECK(hipMemset(ctr, 0, 8));
    hipLaunchKernelGGL(k_count, dim3(1024), dim3(256), 0, 0, p, n, v, ctr, ctr + 1);
    unsigned c[2];
    CHECK(hipMemcpy(c, ctr, 8, hipMemcpyDeviceToHost));
    uint32_t h[2];
    CHECK(hipMemcpy(&h[0], p, 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&h[1], p + n - 1, 4, hipMemcpyDeviceToHost));
    s.rounds++;
    s.kernel_bad += c[0] != 0;
    s.bad_words += c[0];
    s.zero_words += c[1];
    s.dma_bad += (h[0] != v || h[1] != v);
    const uint32_t w = v ^ 0xF0000000u;
    hipLaunchKernelGGL(k_set, dim3(1024), dim3(256), 0, 0, p, n, w);    /* kernel write */
    CHECK(hipMemcpy(&h[0], p, 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&h[1], p + n - 1, 4, hipMemcpyDeviceToHost));
    s.dma_after_kernel_bad += (h[0] != w || h[1] != w);
}

/* ---- multi-process mode ------------------------------------------------- */
static double now_s()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void put_file(const std::string &dir, const std::string &name, const void *p, size_t n)
{
    const std::string tmp = dir + "/." + name + ".tmp", fin = dir + "/" + name;
    FILE *f = fopen(tmp.c_str(), "wb");
    if (f == nullptr || fwrite(p, 1, n, f) != n || fclose(f) != 0 ||
        rename(tmp.c_str(), fin.c_str()) != 0) {
        printf("FAIL put_file %s\n", fin.c_str());
        exit(1);
    }
}

static bool get_file(const std::string &dir, const std::string &name, void *p, size_t n)
{
    FILE *f = fopen((dir + "/" + name).c_str(), "rb");
    if (f == nullptr) {
        return false;
    }
    const size_t r = fread(p, 1, n, f);
    fclose(f);
    return r == n;
}

static void barrier(const std::string &dir, const std::string &tag, int rank, int np)
{
    char one = 1;
    put_file(dir, tag + "_" + std::to_string(rank), &one, 1);
    const double t0 = now_s();
    for (int r = 0; r < np; r++) {
        while (!get_file(dir, tag + "_" + std::to_string(r), &one, 1)) {
            if (now_s() - t0 > 60) {
                printf("FAIL barrier %s timeout waiting for %d\n", tag.c_str(), r);
                exit(1);
            }
            usleep(100);
        }
    }
}

static int ipc_mode(int argc, char **argv)
{
    if (argc < 8) {
        fprintf(stderr, "usage: va_reuse_probe ipc <dir> <rank> <np> <iters> <MiB> <close|hold>\n");
        return 2;
    }
    const std::string dir = argv[2];
    const int rank = atoi(argv[3]), np = atoi(argv[4]), iters = atoi(argv[5]);
    const size_t bytes = (size_t)atoi(argv[6]) << 20, n = bytes / 4;
    const bool hold = strcmp(argv[7], "hold") == 0;
    CHECK(hipSetDevice(0));
    unsigned *ctr;
    CHECK(hipMalloc(&ctr, 8));
    std::vector<uint32_t> host(n);
    auto val = [](int r, int i) { return 0x01000000u * (uint32_t)(r + 1) + (uint32_t)i + 1; };
    long own_bad = 0, own_dma_bad = 0, peer_kernel_bad = 0, peer_dma_bad = 0, same_va = 0;
    long export_fail = 0, import_fail = 0, peer_checked = 0, dup_ptr = 0, bad_and_dup = 0;
    unsigned long long bad_words = 0, zero_words = 0;
    std::vector<std::string> first_bad;
    std::vector<void*> held;                      /* hold: last round's imports */
    void *last = nullptr;
    for (int i = 0; i < iters; i++) {
        void *p;
        CHECK(hipMalloc(&p, bytes));
        same_va += p == last;
        last = p;
        host.assign(n, val(rank, i));
        CHECK(hipMemcpy(p, host.data(), bytes, hipMemcpyHostToDevice));          /* DMA upload */
        CHECK(hipMemset(ctr, 0, 8));
        hipLaunchKernelGGL(k_count, dim3(1024), dim3(256), 0, 0, (const uint32_t*)p, n,
                           val(rank, i), ctr, ctr + 1);
        unsigned c[2];
        CHECK(hipMemcpy(c, ctr, 8, hipMemcpyDeviceToHost));
        own_bad += c[0] != 0;
        uint32_t h2[2];
        CHECK(hipMemcpy(&h2[0], p, 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(&h2[1], (uint32_t*)p + n - 1, 4, hipMemcpyDeviceToHost));
        own_dma_bad += (h2[0] != val(rank, i) || h2[1] != val(rank, i));
        /* a handle of all zero bytes tells the peers this round has no key:
         * the runtime refused the export (counted, not fatal) */
        hipIpcMemHandle_t ih;
        if (hipIpcGetMemHandle(&ih, p) != hipSuccess) {
            (void)hipGetLastError();
            memset(&ih, 0, sizeof(ih));
            export_fail++;
        }
        put_file(dir, "key_" + std::to_string(rank) + "_" + std::to_string(i), &ih, sizeof(ih));
        barrier(dir, "a" + std::to_string(i), rank, np);
        std::vector<void*> maps;
        for (int q = 0; q < np; q++) {
            if (q == rank) continue;
            hipIpcMemHandle_t qh;
            if (!get_file(dir, "key_" + std::to_string(q) + "_" + std::to_string(i), &qh,
                          sizeof(qh))) {
                printf("FAIL key of %d round %d\n", q, i);
                return 1;
            }
            static const hipIpcMemHandle_t none = {};
            if (memcmp(&qh, &none, sizeof(qh)) == 0) {
                continue;                               /* the peer could not export */
            }
            void *m = nullptr;
            if (hipIpcOpenMemHandle(&m, qh, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                (void)hipGetLastError();
                import_fail++;
                continue;
            }
            peer_checked++;
            /* the runtime handed out a mapping this round already has for
             * another peer's handle: the same pointer twice */
            bool dup = false;
            for (void *o : maps) {
                dup = dup || o == m;
            }
            dup_ptr += dup;
            maps.push_back(m);
            CHECK(hipMemset(ctr, 0, 8));
            hipLaunchKernelGGL(k_count, dim3(1024), dim3(256), 0, 0, (const uint32_t*)m, n,
                               val(q, i), ctr, ctr + 1);
            CHECK(hipMemcpy(c, ctr, 8, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(&h2[0], m, 4, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(&h2[1], (uint32_t*)m + n - 1, 4, hipMemcpyDeviceToHost));
            const bool kb = c[0] != 0, db = (h2[0] != val(q, i) || h2[1] != val(q, i));
            bad_and_dup += (kb || db) && dup;
            peer_kernel_bad += kb;
            peer_dma_bad += db;
            bad_words += c[0];
            zero_words += c[1];
            if ((kb || db) && first_bad.size() < 8) {
                char b[160];
                snprintf(b, sizeof(b), "round %d peer %d: kernel %u bad (%u zeros), dma %08x/%08x want %08x",
                         i, q, c[0], c[1], h2[0], h2[1], val(q, i));
                first_bad.push_back(b);
            }
        }
        if (hold) {
            for (void *m : held) CHECK(hipIpcCloseMemHandle(m));   /* a round late */
            held = maps;
        }
        barrier(dir, "b" + std::to_string(i), rank, np);          /* every peer read it */
        if (!hold) {
            for (void *m : maps) CHECK(hipIpcCloseMemHandle(m));
            /* round 6: every peer closed its imports of this buffer before it
             * is freed (without this barrier an exporter could free, and
             * allocate the address again, under a slower peer's open import:
             * the hold mode's hazard) */
            barrier(dir, "c" + std::to_string(i), rank, np);
        }
        CHECK(hipDeviceSynchronize());
        CHECK(hipFree(p));
    }
    for (void *m : held) CHECK(hipIpcCloseMemHandle(m));
    barrier(dir, "end", rank, np);
    printf("{\"rank\": %d, \"np\": %d, \"mode\": \"%s\", \"rounds\": %d, \"same_va\": %ld, "
           "\"own_kernel_bad\": %ld, \"own_dma_bad\": %ld, \"peer_kernel_bad\": %ld, "
           "\"peer_dma_bad\": %ld, \"bad_words\": %llu, \"zero_words\": %llu, "
           "\"export_fail\": %ld, \"import_fail\": %ld, \"peer_checked\": %ld, "
           "\"dup_ptr\": %ld, \"bad_and_dup\": %ld, \"first_bad\": [",
           rank, np, hold ? "hold" : "close", iters, same_va, own_bad, own_dma_bad,
           peer_kernel_bad, peer_dma_bad, bad_words, zero_words, export_fail, import_fail,
           peer_checked, dup_ptr, bad_and_dup);
    for (size_t k = 0; k < first_bad.size(); k++) {
        printf("%s\"%s\"", k ? ", " : "", first_bad[k].c_str());
    }
    printf("]}\n");
    return 0;
}

int main(int argc, char **argv)
{
    setvbuf(stdout, nullptr, _IOLBF, 0);
    if (argc > 1 && strcmp(argv[1], "ipc") == 0) {
        return ipc_mode(argc, argv);
    }
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    const size_t bytes = (size_t)(argc > 2 ? atoi(argv[2]) : 6) << 20, n = bytes / 4;
    CHECK(hipSetDevice(0));
    unsigned *ctr;
    CHECK(hipMalloc(&ctr, 8));
    hipMemAllocationProp pr = prop();
    for (const char *mode : {"same", "fresh", "reserve", "malloc", "same_kcopy", "reserve_kcopy"}) {
        Stats s;
        void *keep = nullptr, *last = nullptr;
        const bool kcopy = strstr(mode, "_kcopy") != nullptr;
        if (!strncmp(mode, "same", 4)) {
            CHECK(hipMemAddressReserve(&keep, bytes, 2 << 20, nullptr, 0));
        }
        for (int i = 0; i < iters; i++) {
            const uint32_t v = 0x10000u + (uint32_t)i;
            if (!strcmp(mode, "malloc")) {
                void *p;
                CHECK(hipMalloc(&p, bytes));
                s.same_va += p == last;
                last = p;
                check_round((uint32_t*)p, n, v, ctr, s);
                CHECK(hipFree(p));
                continue;
            }
            hipMemGenericAllocationHandle_t h;
            CHECK(hipMemCreate(&h, bytes, &pr, 0));
            void *va = keep;
            if (!va) {
                CHECK(hipMemAddressReserve(&va, bytes, 2 << 20, nullptr, 0));
            }
            s.same_va += va == last;
            last = va;
            map_rw(va, bytes, h);
            check_round((uint32_t*)va, n, v, ctr, s, kcopy);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemUnmap(va, bytes));
            CHECK(hipMemRelease(h));
            if (!strncmp(mode, "reserve", 7)) {
                CHECK(hipMemAddressFree(va, bytes));
            }
        }
        printf("%-8s rounds %d, same address as the previous round %d: after the upload (%s), "
               "a kernel saw wrong words in %d rounds (%llu words, %llu zeros) and DMA in %d; "
               "after a kernel write, DMA in %d\n", mode, s.rounds, s.same_va, kcopy ? "kernel" : "DMA", s.kernel_bad,
               s.bad_words, s.zero_words, s.dma_bad, s.dma_after_kernel_bad);
    }
    return 0;
}
