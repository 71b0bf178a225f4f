/*
 * vmm_probe.hip - can peer mappings name physical allocations instead of
 * (pid, address, size)? (VERDICT r03, next #2.) Two processes on one GPU,
 * both started by scripts/vmm_probe.py (a parent that never touches the GPU):
 *
 *   vmm_probe export <socket name> <MiB>   creates a VMM allocation
 *        (hipMemCreate, POSIX fd handle type), fills it, exports the fd
 *        (hipMemExportToShareableHandle) and passes it over a Unix socket
 *        (SCM_RIGHTS); then frees it, makes a new one of the same size at the
 *        same reserved address with other contents, and passes that one
 *   vmm_probe import <socket name> <MiB>   imports each fd
 *        (hipMemImportFromShareableHandle + hipMemMap), checks the contents
 *        by DMA and by a kernel, writes its mark into the second half, and
 *        reports; also tries pidfd_getfd on the exporter's fd
 *
 * Also reported: what the runtime says about a VMM pointer (address range,
 * buffer id, legacy IPC handle), and the 2 x 256 MiB fp32 combine
 * (k_reduce) on hipMalloc memory vs VMM memory, one and two allocations.
 * Built by `make -C tools/src` into tools/ (not part of the product).
 */
#include <hip/hip_runtime.h>

#include <sys/socket.h>
#include <sys/syscall.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <tuple>
#include <vector>

#include "dev_kernels.h"

using namespace ucgdev;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("FAIL %s: %s\n", #x, hipGetErrorString(e_)); fflush(stdout); exit(1); } } while (0)

static int sock_addr(const char *name, sockaddr_un *a)
{
    memset(a, 0, sizeof(*a));
    a->sun_family = AF_UNIX;
    a->sun_path[0] = '\0';                      /* abstract namespace */
    snprintf(a->sun_path + 1, sizeof(a->sun_path) - 1, "%s", name);
    return (int)(offsetof(sockaddr_un, sun_path) + 1 + strlen(name));
}

struct Msg {
    uint64_t size, gen, pid;
    int      fd_num;      /* the exporter's own fd number (for pidfd_getfd) */
};

static int send_fd(int s, int fd, const Msg &m)
{
    char cbuf[CMSG_SPACE(sizeof(int))];
    memset(cbuf, 0, sizeof(cbuf));
    iovec iov = {(void*)&m, sizeof(m)};
    msghdr mh = {};
    mh.msg_iov = &iov;
    mh.msg_iovlen = 1;
    mh.msg_control = cbuf;
    mh.msg_controllen = sizeof(cbuf);
    cmsghdr *c = CMSG_FIRSTHDR(&mh);
    c->cmsg_level = SOL_SOCKET;
    c->cmsg_type = SCM_RIGHTS;
    c->cmsg_len = CMSG_LEN(sizeof(int));
    memcpy(CMSG_DATA(c), &fd, sizeof(int));
    return sendmsg(s, &mh, 0) == (ssize_t)sizeof(m) ? 0 : -1;
}

static int recv_fd(int s, Msg *m)
{
    char cbuf[CMSG_SPACE(sizeof(int))];
    iovec iov = {(void*)m, sizeof(*m)};
    msghdr mh = {};
    mh.msg_iov = &iov;
    mh.msg_iovlen = 1;
    mh.msg_control = cbuf;
    mh.msg_controllen = sizeof(cbuf);
    if (recvmsg(s, &mh, MSG_WAITALL) != (ssize_t)sizeof(*m)) {
        return -1;
    }
    cmsghdr *c = CMSG_FIRSTHDR(&mh);
    if (!c || c->cmsg_type != SCM_RIGHTS) {
        return -1;
    }
    int fd;
    memcpy(&fd, CMSG_DATA(c), sizeof(int));
    return fd;
}

static hipMemAllocationProp prop_for(int dev)
{
    hipMemAllocationProp p = {};
    p.type = hipMemAllocationTypePinned;
    p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = dev;
    return p;
}

static void map_rw(void *va, size_t size, hipMemGenericAllocationHandle_t h, int dev)
{
    CHECK(hipMemMap(va, size, 0, h, 0));
    hipMemAccessDesc d = {};
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = dev;
    d.flags = hipMemAccessFlagsProtReadWrite;
    CHECK(hipMemSetAccess(va, size, &d, 1));
}

/* words of the pattern: key ^ index */
__global__ void k_pattern(uint32_t *p, size_t n, uint32_t key)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        p[i] = key ^ (uint32_t)i;
    }
}

__global__ void k_check(const uint32_t *p, size_t n, uint32_t key, unsigned *bad)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        if (p[i] != (key ^ (uint32_t)i)) {
            atomicAdd(bad, 1u);
        }
    }
}

static size_t host_bad(const uint32_t *dev, size_t n, uint32_t key)
{
    std::vector<uint32_t> h(n);
    CHECK(hipMemcpy(h.data(), dev, n * 4, hipMemcpyDeviceToHost));
    size_t b = 0;
    for (size_t i = 0; i < n; i++) {
        b += h[i] != (key ^ (uint32_t)i);
    }
    return b;
}

static unsigned kernel_bad(const uint32_t *p, size_t n, uint32_t key)
{
    unsigned *bad;
    CHECK(hipMalloc(&bad, 4));
    CHECK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, 0, p, n, key, bad);
    unsigned b = 0;
    CHECK(hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost));
    CHECK(hipFree(bad));
    return b;
}

static double now_s()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* k_reduce (the product geometry) on dst/src, median of 5 batches of 20 */
static double combine_pct(float *d, const float *s, size_t n)
{
    const size_t nvec = n / 4;
    const unsigned g = (unsigned)(nvec / kReduceBlock);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<float> us;
    for (int r = 0; r < 6; r++) {
        CHECK(hipEventRecord(e0, 0));
        for (int i = 0; i < 20; i++) {
            hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock>), dim3(g),
                               dim3(kReduceBlock), 0, 0, d, s, (size_t)0, nvec, (size_t)0);
        }
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (r) us.push_back(1000.f * ms / 20);
    }
    std::sort(us.begin(), us.end());
    return 100.0 * 3.0 * n * 4 / (us[us.size() / 2] * 1e-6) / 8e12;
}

static void *vmm_alloc(size_t bytes, hipMemGenericAllocationHandle_t *h, size_t gran,
                       size_t align = 0)
{
    hipMemAllocationProp p = prop_for(0);
    bytes = (bytes + gran - 1) / gran * gran;
    CHECK(hipMemCreate(h, bytes, &p, 0));
    void *va = nullptr;
    CHECK(hipMemAddressReserve(&va, bytes, align ? align : gran, nullptr, 0));
    map_rw(va, bytes, *h, 0);
    return va;
}

static int do_export(const char *name, size_t mib)
{
    CHECK(hipSetDevice(0));
    int vmm = 0;
    CHECK(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, 0));
    hipMemAllocationProp prop = prop_for(0);
    size_t gran = 0, rgran = 0;
    CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    CHECK(hipMemGetAllocationGranularity(&rgran, &prop, hipMemAllocationGranularityRecommended));
    printf("export: vmm supported %d, granularity min %zu recommended %zu\n", vmm, gran, rgran);
    const size_t bytes = mib << 20, n = bytes / 4;

    double t0 = now_s();
    hipMemGenericAllocationHandle_t h;
    CHECK(hipMemCreate(&h, bytes, &prop, 0));
    void *va = nullptr;
    CHECK(hipMemAddressReserve(&va, bytes, gran, nullptr, 0));
    map_rw(va, bytes, h, 0);
    printf("export: create+reserve+map+access %.3f ms at %p\n", (now_s() - t0) * 1e3, va);

    /* what the runtime says about a VMM pointer */
    hipDeviceptr_t base = nullptr;
    size_t rsize = 0;
    hipError_t e = hipMemGetAddressRange(&base, &rsize, (hipDeviceptr_t)((char*)va + 4096));
    printf("export: hipMemGetAddressRange(va+4096) %s base %p size %zu\n", hipGetErrorString(e),
           (void*)base, rsize);
    unsigned long long bid = 0;
    e = hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)va);
    printf("export: buffer id %s %llu\n", hipGetErrorString(e), bid);
    hipIpcMemHandle_t ih;
    e = hipIpcGetMemHandle(&ih, va);
    printf("export: hipIpcGetMemHandle on VMM memory: %s\n", hipGetErrorString(e));
    (void)hipGetLastError();
    {
        void *pm = nullptr;
        CHECK(hipMalloc(&pm, 2 << 20));
        unsigned long long b1 = 0, b2 = 0;
        (void)hipPointerGetAttribute(&b1, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)pm);
        CHECK(hipFree(pm));
        void *pm2 = nullptr;
        CHECK(hipMalloc(&pm2, 2 << 20));
        e = hipPointerGetAttribute(&b2, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)pm2);
        printf("export: hipMalloc buffer ids across free+malloc: %llu -> %llu (%s), same address %d\n",
               b1, b2, hipGetErrorString(e), (int)(pm == pm2));
        CHECK(hipFree(pm2));
    }

    hipLaunchKernelGGL(k_pattern, dim3(1024), dim3(256), 0, 0, (uint32_t*)va, n, 0xA0000000u);
    CHECK(hipDeviceSynchronize());

    int fd = -1;
    t0 = now_s();
    CHECK(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0));
    printf("export: fd %d (%.3f ms)\n", fd, (now_s() - t0) * 1e3);

    int ls = socket(AF_UNIX, SOCK_STREAM, 0);
    sockaddr_un a;
    const int alen = sock_addr(name, &a);
    if (bind(ls, (sockaddr*)&a, alen) || listen(ls, 1)) {
        printf("FAIL bind/listen: %s\n", strerror(errno));
        return 1;
    }
    printf("export: listening\n");
    fflush(stdout);
    int s = accept(ls, nullptr, nullptr);
    Msg m = {bytes, 1, (uint64_t)getpid(), fd};
    if (send_fd(s, fd, m)) {
        printf("FAIL send_fd: %s\n", strerror(errno));
        return 1;
    }
    char ack[8];
    if (read(s, ack, 4) != 4) {
        printf("FAIL no ack\n");
        return 1;
    }
    /* the importer wrote its mark into the second half */
    printf("export: importer's mark seen by the exporter: %zu bad words, first half %zu\n",
           host_bad((uint32_t*)va + n / 2, n / 2, 0xB0000000u),
           host_bad((uint32_t*)va, n / 2, 0xA0000000u));

    /* free it, make a new allocation at the same reserved range, other data */
    close(fd);
    CHECK(hipMemUnmap(va, bytes));
    CHECK(hipMemRelease(h));
    hipMemGenericAllocationHandle_t h2;
    CHECK(hipMemCreate(&h2, bytes, &prop, 0));
    map_rw(va, bytes, h2, 0);
    hipLaunchKernelGGL(k_pattern, dim3(1024), dim3(256), 0, 0, (uint32_t*)va, n, 0xC0000000u);
    CHECK(hipDeviceSynchronize());
    int fd2 = -1;
    CHECK(hipMemExportToShareableHandle(&fd2, h2, hipMemHandleTypePosixFileDescriptor, 0));
    Msg m2 = {bytes, 2, (uint64_t)getpid(), fd2};
    send_fd(s, fd2, m2);
    if (read(s, ack, 4) != 4) {
        printf("FAIL no second ack\n");
        return 1;
    }
    close(fd2);
    close(s);
    close(ls);
    CHECK(hipMemUnmap(va, bytes));
    CHECK(hipMemRelease(h2));
    CHECK(hipMemAddressFree(va, bytes));

    /* the combine on hipMalloc memory vs VMM memory */
    const size_t cn = (size_t)1 << 26;
    {
        float *pair;
        CHECK(hipMalloc(&pair, 2 * cn * 4));
        float *a1, *a2;
        CHECK(hipMalloc(&a1, cn * 4));
        CHECK(hipMalloc(&a2, cn * 4));
        hipMemGenericAllocationHandle_t hp, h1, h2b;
        float *vpair = (float*)vmm_alloc(2 * cn * 4, &hp, gran);
        float *v1 = (float*)vmm_alloc(cn * 4, &h1, gran);
        float *v2 = (float*)vmm_alloc(cn * 4, &h2b, gran);
        for (float *p : {pair, pair + cn, a1, a2, vpair, vpair + cn, v1, v2}) {
            hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                               (void*)p, 1, (uint64_t)(uintptr_t)p, cn);
        }
        CHECK(hipDeviceSynchronize());
        for (int r = 0; r < 3; r++) {
            printf("combine 2 x 256 MiB fp32, %% of 8 TB/s: hipMalloc one allocation %.1f, "
                   "two %.1f; VMM one %.1f, two %.1f\n",
                   combine_pct(pair + cn, pair, cn), combine_pct(a2, a1, cn),
                   combine_pct(vpair + cn, vpair, cn), combine_pct(v2, v1, cn));
        }
    }
    printf("export: ok\n");
    return 0;
}

__global__ void k_nop(unsigned *p)
{
    if (p != nullptr && threadIdx.x == 1024) {
        p[0] = 1;                          /* never: keeps the kernel non-empty */
    }
}

__global__ void k_sum(const uint32_t *p, size_t n, unsigned *out)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        acc += p[i];
    }
    if (acc == 0x12345678u) {
        out[0] = acc;                      /* practically never: keeps the loads */
    }
}

/* average time per launch of `fn` over `reps` back-to-back launches (us) */
template <typename F>
static double per_launch_us(F fn, int reps)
{
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    fn();
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; i++) {
        fn();
    }
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return 1000.0 * ms / reps;
}

/* round 4: kernels reading imported VMM memory ran 5-10x longer
 * in the engine. What costs: any kernel once an import is mapped, or only
 * the ones that read it? An empty kernel, a 4 KiB read and a 64 MiB read, on
 * the import, on this process's own hipMalloc memory and on its own VMM
 * memory. */
static void import_costs(const char *when, const uint32_t *imp, size_t n, const uint32_t *own,
                         const uint32_t *own_vmm, unsigned *ctr)
{
    const int reps = 2000;
    printf("import cost %s: empty kernel %.2f us", when,
           per_launch_us([&] { hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, 0, ctr); }, reps));
    if (imp == nullptr) {
        printf("\n");
        return;
    }
    auto rd = [&](const uint32_t *p, size_t words, unsigned grid) {
        return per_launch_us([&] { hipLaunchKernelGGL(k_sum, dim3(grid), dim3(256), 0, 0, p,
                                                      words, ctr); }, words > 4096 ? 50 : reps);
    };
    printf("; 4 KiB read: import %.2f us, own hipMalloc %.2f us, own VMM %.2f us",
           rd(imp, 1024, 4), rd(own, 1024, 4), rd(own_vmm, 1024, 4));
    printf("; %zu MiB read: import %.1f us, own hipMalloc %.1f us, own VMM %.1f us\n",
           n * 4 >> 20, rd(imp, n, 4096), rd(own, n, 4096), rd(own_vmm, n, 4096));
}

static int do_import(const char *name, size_t mib)
{
    CHECK(hipSetDevice(0));
    const size_t bytes = mib << 20, n = bytes / 4;
    unsigned *ctr;
    uint32_t *own;
    CHECK(hipMalloc(&ctr, 64));
    CHECK(hipMalloc(&own, bytes));
    CHECK(hipMemset(own, 1, bytes));
    import_costs("before any import", nullptr, 0, nullptr, nullptr, ctr);
    hipMemAllocationProp prop = prop_for(0);
    size_t gran = 0;
    CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    int s = socket(AF_UNIX, SOCK_STREAM, 0);
    sockaddr_un a;
    const int alen = sock_addr(name, &a);
    int tries = 0;
    while (connect(s, (sockaddr*)&a, alen) != 0) {
        if (++tries > 600) {
            printf("FAIL connect: %s\n", strerror(errno));
            return 1;
        }
        usleep(50000);
    }
    for (int round = 0; round < 2; round++) {
        Msg m;
        const int fd = recv_fd(s, &m);
        if (fd < 0) {
            printf("FAIL recv_fd\n");
            return 1;
        }
        if (round == 0) {
            /* the alternative to SCM_RIGHTS: take the fd from the exporter */
            int pfd = (int)syscall(SYS_pidfd_open, (pid_t)m.pid, 0);
            int got = pfd >= 0 ? (int)syscall(SYS_pidfd_getfd, pfd, m.fd_num, 0) : -1;
            printf("import: pidfd_open %s, pidfd_getfd %s\n", pfd >= 0 ? "ok" : strerror(errno),
                   got >= 0 ? "ok" : strerror(errno));
            if (got >= 0) close(got);
            if (pfd >= 0) close(pfd);
        }
        double t0 = now_s();
        hipMemGenericAllocationHandle_t h;
        /* VMM_FD_CONV=pointer: pass the address of the fd, not its value */
        const char *conv = getenv("VMM_FD_CONV");
        int fdv = fd;
        int rtv = 0;
        (void)hipRuntimeGetVersion(&rtv);
        printf("import: runtime %d, fd convention %s\n", rtv, conv ? conv : "value");
        CHECK(hipMemImportFromShareableHandle(&h, (conv && conv[0] == 'p') ? (void*)&fdv
                                                  : (void*)(intptr_t)fd,
                                              hipMemHandleTypePosixFileDescriptor));
        void *va = nullptr;
        CHECK(hipMemAddressReserve(&va, m.size, gran, nullptr, 0));
        map_rw(va, m.size, h, 0);
        const double ms = (now_s() - t0) * 1e3;
        const uint32_t key = round == 0 ? 0xA0000000u : 0xC0000000u;
        printf("import gen %llu: import+map %.3f ms at %p; bad words by DMA %zu, by kernel %u\n",
               (unsigned long long)m.gen, ms, va, host_bad((uint32_t*)va, n, key),
               kernel_bad((uint32_t*)va, n, key));
        if (round == 0) {
            hipMemGenericAllocationHandle_t hv;
            void *ov = nullptr;
            CHECK(hipMemCreate(&hv, bytes, &prop, 0));
            CHECK(hipMemAddressReserve(&ov, bytes, gran, nullptr, 0));
            map_rw(ov, bytes, hv, 0);
            CHECK(hipMemset(ov, 1, bytes));
            CHECK(hipDeviceSynchronize());
            import_costs("with the import mapped", (const uint32_t*)va, n, own,
                         (const uint32_t*)ov, ctr);
            hipLaunchKernelGGL(k_pattern, dim3(1024), dim3(256), 0, 0, (uint32_t*)va + n / 2,
                               n / 2, 0xB0000000u);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemUnmap(ov, bytes));
            CHECK(hipMemRelease(hv));
            CHECK(hipMemAddressFree(ov, bytes));
        }
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemUnmap(va, m.size));
        CHECK(hipMemRelease(h));
        CHECK(hipMemAddressFree(va, m.size));
        close(fd);
        if (write(s, "ack!", 4) != 4) {
            printf("FAIL ack\n");
            return 1;
        }
    }
    close(s);
    import_costs("after the imports were released", nullptr, 0, nullptr, nullptr, ctr);
    CHECK(hipFree(own));
    CHECK(hipFree(ctr));
    printf("import: ok\n");
    return 0;
}

/* the combine on VMM memory reserved at several alignments */
static int do_perf()
{
    CHECK(hipSetDevice(0));
    hipMemAllocationProp prop = prop_for(0);
    size_t gran = 0;
    CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    const size_t cn = (size_t)1 << 26;
    float *pair, *a1, *a2;
    CHECK(hipMalloc(&pair, 2 * cn * 4));
    CHECK(hipMalloc(&a1, cn * 4));
    CHECK(hipMalloc(&a2, cn * 4));
    printf("hipMalloc pair at %p, separate at %p %p\n", (void*)pair, (void*)a1, (void*)a2);
    for (size_t align : {(size_t)4096, (size_t)2 << 20, (size_t)64 << 20, (size_t)1 << 30}) {
        hipMemGenericAllocationHandle_t hp, h1, h2;
        double t0 = now_s();
        float *vp = (float*)vmm_alloc(2 * cn * 4, &hp, gran, align);
        const double ms = (now_s() - t0) * 1e3;
        float *v1 = (float*)vmm_alloc(cn * 4, &h1, gran, align);
        float *v2 = (float*)vmm_alloc(cn * 4, &h2, gran, align);
        for (float *p : {pair, pair + cn, a1, a2, vp, vp + cn, v1, v2}) {
            hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                               (void*)p, 1, (uint64_t)(uintptr_t)p, cn);
        }
        CHECK(hipDeviceSynchronize());
        for (int r = 0; r < 2; r++) {
            printf("align %10zu (512 MiB create+map %.1f ms): %% of 8 TB/s hipMalloc one %.1f "
                   "two %.1f | VMM one %.1f two %.1f\n", align, ms,
                   combine_pct(pair + cn, pair, cn), combine_pct(a2, a1, cn),
                   combine_pct(vp + cn, vp, cn), combine_pct(v2, v1, cn));
        }
        for (auto [p, h, b] : {std::make_tuple((void*)vp, hp, 2 * cn * 4),
                               std::make_tuple((void*)v1, h1, cn * 4),
                               std::make_tuple((void*)v2, h2, cn * 4)}) {
            CHECK(hipMemUnmap(p, b));
            CHECK(hipMemRelease(h));
            CHECK(hipMemAddressFree(p, b));
        }
    }
    return 0;
}

int main(int argc, char **argv)
{
    if (argc > 1 && strcmp(argv[1], "perf") == 0) {
        setvbuf(stdout, nullptr, _IOLBF, 0);
        return do_perf();
    }
    if (argc < 4) {
        fprintf(stderr, "usage: vmm_probe export|import <socket name> <MiB>\n");
        return 2;
    }
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const size_t mib = (size_t)atoll(argv[3]);
    return strcmp(argv[1], "export") == 0 ? do_export(argv[2], mib) : do_import(argv[2], mib);
}
