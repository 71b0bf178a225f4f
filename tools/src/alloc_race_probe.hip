/*
 * alloc_race_probe.hip - does a freshly allocated device buffer keep what was
 * written into it, when many processes allocate and free on one GPU?
 *
 * The worker of the device-buffer engine tests (tests/_worker_topo.py) found
 * per-case buffers whose whole allocation - guard zones included - read as
 * zeros some time after an upload that had been read back correctly, before
 * any engine call touched them (profiles/r03/r03s2b). This probe does the same
 * allocation pattern with no engine at all: per iteration, allocate two
 * buffers (2 MiB granules, as ucg_builtin_dev_malloc rounds), upload a
 * pattern, read it back, run a small kernel that reads one and writes the
 * other, read both back again, free both. Optionally (mode "ipc") every
 * process also exports a long-lived buffer and imports every peer's, as the
 * engine's pools do, and a kernel reads the imports each iteration.
 *
 *   alloc_race_probe <rank> <nprocs> <iters> <mode: plain|ipc|lds> <shm-dir>
 *
 * Mode "lds" (no IPC) adds what the engine did when the zeroed allocations
 * were most frequent: each iteration also launches small kernels with
 * 20 KiB of dynamic LDS they never touch on four streams of the process.
 *
 * Prints one line: iterations, buffers whose content changed after the
 * verified upload (and how many of those read as all zeros).
 * Built by `make -C tools/src` into tools/ (not part of the product).
 */
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

/* a few workgroups holding dynamic LDS they never touch (the occupancy cap's
 * launches on small grids) */
__global__ void k_small(uint32_t *out, const uint32_t *in, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        out[i] = in[i] ^ 0x5a5a5a5au;
    }
}

__global__ void k_touch(uint32_t *out, const uint32_t *in, size_t n, const uint32_t *peer,
                        size_t pn)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint32_t v = in[i];
        if (peer && i < pn) {
            v += (peer[i] == 0xDEADBEEFu);   /* a real read of the peer mapping (0x11 bytes: adds 0) */
        }
        out[i] = v + 1;
    }
}

static void fill(std::vector<uint32_t> &h, uint32_t seed)
{
    for (size_t i = 0; i < h.size(); i++) {
        h[i] = (uint32_t)(i * 2654435761u) ^ seed ^ 0xA5A5A5A5u;
    }
}

int main(int argc, char **argv)
{
    if (argc < 6) {
        fprintf(stderr, "usage: %s rank nprocs iters plain|ipc shm-dir\n", argv[0]);
        return 2;
    }
    const int rank = atoi(argv[1]), nprocs = atoi(argv[2]), iters = atoi(argv[3]);
    const bool ipc = strcmp(argv[4], "ipc") == 0;
    const bool lds = strcmp(argv[4], "lds") == 0;
    const std::string dir = argv[5];
    const size_t bytes = (size_t)2 << 20;           /* one 2 MiB granule */
    const size_t n = bytes / 4;

    /* ipc: a long-lived exported buffer per process, every peer's imported */
    std::vector<void*> peers;
    uint32_t *mine = nullptr;
    if (ipc) {
        CHECK(hipMalloc(&mine, bytes));
        CHECK(hipMemset(mine, 0x11, bytes));
        hipIpcMemHandle_t h;
        CHECK(hipIpcGetMemHandle(&h, mine));
        const std::string f = dir + "/h" + std::to_string(rank);
        FILE *fp = fopen((f + ".tmp").c_str(), "wb");
        fwrite(&h, sizeof(h), 1, fp);
        fclose(fp);
        rename((f + ".tmp").c_str(), f.c_str());
        for (int r = 0; r < nprocs; r++) {
            if (r == rank) continue;
            const std::string g = dir + "/h" + std::to_string(r);
            FILE *q = nullptr;
            for (int t = 0; t < 6000 && !(q = fopen(g.c_str(), "rb")); t++) {
                std::this_thread::sleep_for(std::chrono::milliseconds(10));
            }
            if (!q) { fprintf(stderr, "rank %d: no handle from %d\n", rank, r); return 1; }
            hipIpcMemHandle_t ph;
            if (fread(&ph, sizeof(ph), 1, q) != 1) { fclose(q); return 1; }
            fclose(q);
            void *p = nullptr;
            CHECK(hipIpcOpenMemHandle(&p, ph, hipIpcMemLazyEnablePeerAccess));
            peers.push_back(p);
        }
    }

    std::vector<uint32_t> pat(n), got(n);
    size_t changed = 0, zeros = 0, checked = 0, upload_lost = 0;
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipStream_t side[4];
    uint32_t *scratch = nullptr;
    if (lds) {
        for (auto &q : side) {
            CHECK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
        }
        CHECK(hipMalloc(&scratch, 4 * 4096 * sizeof(uint32_t)));
    }
    for (int it = 0; it < iters; it++) {
        uint32_t *a = nullptr, *b = nullptr;
        CHECK(hipMalloc(&a, bytes));
        CHECK(hipMalloc(&b, bytes));
        fill(pat, (uint32_t)(rank * 1000003 + it));
        CHECK(hipMemcpy(a, pat.data(), bytes, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(got.data(), a, bytes, hipMemcpyDeviceToHost));
        if (memcmp(got.data(), pat.data(), bytes) != 0) {
            upload_lost++;
        }
        const uint32_t *pp = peers.empty() ? nullptr
                           : static_cast<const uint32_t*>(peers[it % peers.size()]);
        hipLaunchKernelGGL(k_touch, dim3((unsigned)(n / 256)), dim3(256), 0, st, b, a, n,
                           pp, n);
        if (lds) {
            for (int k = 0; k < 4; k++) {
                hipLaunchKernelGGL(k_small, dim3(4), dim3(64), 20480, side[k],
                                   scratch + k * 4096, a + k * 4096, (size_t)256);
            }
            for (auto &q : side) {
                CHECK(hipStreamSynchronize(q));
            }
        }
        CHECK(hipStreamSynchronize(st));
        /* a pause of 0-2 ms, as a test process has between upload and use */
        std::this_thread::sleep_for(std::chrono::microseconds((it * 7919 + rank * 104729) % 2000));
        CHECK(hipMemcpy(got.data(), a, bytes, hipMemcpyDeviceToHost));
        checked++;
        if (memcmp(got.data(), pat.data(), bytes) != 0) {
            changed++;
            size_t z = 0;
            for (size_t i = 0; i < n; i++) z += got[i] == 0;
            if (z == n) zeros++;
            fprintf(stderr, "rank %d iter %d: buffer at %p changed after a verified upload "
                    "(%zu of %zu words zero)\n", rank, it, (void*)a, z, n);
        }
        CHECK(hipFree(a));
        CHECK(hipFree(b));
    }
    for (void *p : peers) {
        CHECK(hipIpcCloseMemHandle(p));
    }
    printf("rank %d mode %s iters %d checked %zu changed %zu all_zero %zu upload_lost %zu\n",
           rank, argv[4], iters, checked, changed, zeros, upload_lost);
    if (scratch) {
        CHECK(hipFree(scratch));
    }
    if (mine) {
        /* peers may still hold the mapping: wait for them before freeing */
        const std::string f = dir + "/done" + std::to_string(rank);
        FILE *fp = fopen(f.c_str(), "wb");
        fclose(fp);
        for (int r = 0; r < nprocs; r++) {
            const std::string g = dir + "/done" + std::to_string(r);
            for (int t = 0; t < 6000; t++) {
                FILE *q = fopen(g.c_str(), "rb");
                if (q) { fclose(q); break; }
                std::this_thread::sleep_for(std::chrono::milliseconds(10));
            }
        }
        CHECK(hipFree(mine));
    }
    return changed ? 4 : 0;
}
