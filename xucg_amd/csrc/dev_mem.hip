/*
 * dev_mem.hip - device memory and peer mapping of the C-ABI shim
 * (include/ucg_builtin_dev.h, "peer mapping" and "memory helpers").
 *
 * It stands in for the memory registration and remote keys the reference gets
 * from UCT (uct_md_mem_reg / uct_md_mkey_pack for the zero-copy steps,
 * builtin/ops/builtin_control.c:276-286, 712-719, 1284-1304): a key names a
 * buffer so that a peer process can read it in place, over xGMI.
 *
 * A key names a physical allocation, never an address (round 4):
 *  - Shareable allocations (ucg_builtin_dev_malloc_shareable) are HIP virtual
 *    memory: hipMemCreate with a POSIX file descriptor handle type, mapped at
 *    a reservation of this process. A peer maps one from its file
 *    descriptor, which it gets from the exporter's key server over a Unix
 *    socket (SCM_RIGHTS): the fd holds the physical memory itself, so a key
 *    can never resolve to another allocation, and a peer's mapping keeps the
 *    memory alive after the exporter frees it (no fault, and nobody else's
 *    data).
 *  - Other device memory (ucg_builtin_dev_malloc, a caller's hipMalloc) is
 *    exported with hipIpcGetMemHandle, whose handle names (pid, address,
 *    size). The key server hands that handle out only while the runtime's
 *    buffer id of the allocation at that address is the one recorded at
 *    export: a buffer freed and allocated again at the same address is a new
 *    allocation, and its old keys are refused.
 * Every key carries a per-process id that is never reused; freeing an
 * exported allocation retires its id, so a stale key fails loudly at import
 * (UCS_ERR_NO_RESOURCE, "stale key") instead of mapping
 * whatever now lives there. This replaces round 3's rule that exported
 * memory is never freed (stale IPC keys).
 */
#include <hip/hip_runtime.h>

#include <execinfo.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <fcntl.h>
#include <pthread.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "dev_internal.h"

namespace {

constexpr size_t kGran = (size_t)2 << 20;     /* allocation and mapping granule */

size_t round_gran(size_t bytes)
{
    return bytes ? (bytes + kGran - 1) / kGran * kGran : kGran;
}

/* ---- the process's allocations and memory events ------------------------- */
enum { KIND_PLAIN = 1, KIND_VMM = 2 };

struct own_alloc {
    int      kind;
    int      device;
    size_t   bytes;
    hipMemGenericAllocationHandle_t handle;   /* KIND_VMM */
    uint64_t key_id;                          /* 0: never exported */
    bool     exported;                        /* KIND_PLAIN: ever exported */
    size_t   want;                            /* bytes the caller asked for (rounded) */
};

std::mutex g_mu;                                      /* guards everything here */
std::unordered_map<void*, own_alloc> g_allocs;        /* base -> allocation */

/* Freed plain allocations kept for reuse at the same size (round 4). A
 * hipFree + hipMalloc can hand out the old address backed by new memory,
 * and the copy engine can then write through the old translation (DESIGN.md
 * 7, tools/va_reuse_probe). Reusing the allocation itself - same address,
 * same memory - never remaps anything. Its keys are retired at free all the
 * same (a peer's old key is refused), and the device is synchronised before
 * it is handed out again. Never-exported allocations are bounded by
 * UCX_BUILTIN_DEV_CACHE_BYTES (default 1 GiB per process; 0 = free at once)
 * and freed past the bound; an allocation that was ever exported is always
 * kept (round 5: given back to the runtime, its address returns with other
 * memory, and peers' fresh hipIpc imports of it can map another process's
 * memory). The value is (pointer, ever exported). */
std::multimap<std::pair<int, size_t>, std::pair<void*, bool>> g_plain_cache;  /* (device, bytes) */
size_t g_plain_cached = 0;       /* never-exported bytes in the cache (bounded) */
size_t g_cached_exported = 0;    /* ever-exported bytes in the cache (kept) */
uint64_t g_parked = 0;           /* bytes parked by ucg_builtin_dev_park */
/* Memory this process keeps for its life (round 6): every
 * ever-exported plain allocation, live or cached, plus what is parked.
 * Bounded by UCX_BUILTIN_DEV_KEEP_MAX (default half the device's memory):
 * exporting an allocation that would take it past the cap fails with
 * UCS_ERR_EXCEEDS_LIMIT, named; half-way there a warning is printed once. */
uint64_t g_kept = 0;
std::atomic<uint64_t> g_keep_max_set{0};          /* 0: the environment's / default */
bool g_keep_warned = false;
/* bytes of live allocations beyond their request: an ever-exported
 * allocation handed out whole for a request of at least half its size */
uint64_t g_slack = 0;

uint64_t parse_bytes(const char *e, uint64_t dflt)
{
    if (e == nullptr || *e == 0) {
        return dflt;
    }
    char *end = nullptr;
    double v = strtod(e, &end);
    if (end && (*end == 'k' || *end == 'K')) v *= 1024.0;
    else if (end && (*end == 'm' || *end == 'M')) v *= 1048576.0;
    else if (end && (*end == 'g' || *end == 'G')) v *= 1073741824.0;
    else if (end && (*end == 't' || *end == 'T')) v *= 1099511627776.0;
    return v > 0 ? (uint64_t)v : dflt;
}

/* the cap on g_kept: ucg_builtin_dev_set_keep_max, else
 * UCX_BUILTIN_DEV_KEEP_MAX, else half of `device`'s memory */
uint64_t keep_max(int device)
{
    const uint64_t set = g_keep_max_set.load(std::memory_order_relaxed);
    if (set) {
        return set;
    }
    static std::atomic<uint64_t> lim{0};
    uint64_t v = lim.load(std::memory_order_relaxed);
    if (v == 0) {
        size_t total = 0;
        if (hipDeviceTotalMem(&total, device) != hipSuccess || total == 0) {
            (void)hipGetLastError();
            total = (size_t)256 << 30;
        }
        v = parse_bytes(getenv("UCX_BUILTIN_DEV_KEEP_MAX"), (uint64_t)total / 2);
        lim.store(v, std::memory_order_relaxed);
    }
    return v;
}

size_t plain_cache_limit()
{
    static const size_t lim = [] {
        const char *e = getenv("UCX_BUILTIN_DEV_CACHE_BYTES");
        if (e == nullptr || *e == 0) {
            return (size_t)1 << 30;
        }
        char *end = nullptr;
        double v = strtod(e, &end);
        if (end && (*end == 'k' || *end == 'K')) v *= 1024.0;
        else if (end && (*end == 'm' || *end == 'M')) v *= 1048576.0;
        else if (end && (*end == 'g' || *end == 'G')) v *= 1073741824.0;
        return v > 0 ? (size_t)v : (size_t)0;
    }();
    return lim;
}

/* give `device`'s never-exported cached allocations back to the runtime
 * (hipMalloc ran out of memory there: the cache may hold what it needs, at
 * other sizes); returns how many. The calling thread's current device is
 * `device` on return (a retried hipMalloc on the device drained
 * last could land on the wrong GPU). Caller does not hold g_mu. */
size_t plain_cache_drain(int device)
{
    std::vector<void*> out;
    {
        std::lock_guard<std::mutex> g(g_mu);
        for (auto it = g_plain_cache.lower_bound({device, 0});
             it != g_plain_cache.end() && it->first.first == device;) {
            if (!it->second.second) {
                out.push_back(it->second.first);
                g_plain_cached -= it->first.second;
                it = g_plain_cache.erase(it);
            } else {
                ++it;
            }
        }
    }
    (void)hipSetDevice(device);
    for (void *p : out) {
        (void)hipFree(p);
    }
    return out.size();
}

/* The last memory events of the process, for ucg_builtin_dev_debug_ptr: a
 * buffer found to read as zeros is matched against what happened to its
 * address range. */
struct mem_event {
    char     kind;      /* M malloc, R malloc from the reuse cache, V shareable malloc, F free, X export,
                           I import, C release (close), S stale key refused, P parked */
    void    *ptr;
    void    *base;
    size_t   bytes;
    uint64_t ns;        /* CLOCK_MONOTONIC */
    int      rc;        /* the runtime's return code */
};
constexpr size_t kMemEvents = 1024;
mem_event g_events[kMemEvents];
uint64_t  g_nevents;

uint64_t now_ns()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

/* caller holds g_mu */
void note_event(char kind, void *ptr, void *base, size_t bytes, int rc)
{
    g_events[g_nevents++ % kMemEvents] = mem_event{kind, ptr, base, bytes, now_ns(), rc};
}

/* ---- exported allocations (the key server's table) ----------------------- */
struct export_rec {
    int                kind;
    void              *base;
    size_t             size;
    int                fd;          /* KIND_VMM: the shareable handle, open while exported */
    unsigned long long buffer_id;   /* KIND_PLAIN: the runtime's id at export */
    hipIpcMemHandle_t  ih;          /* KIND_PLAIN */
};
std::unordered_map<uint64_t, export_rec> g_exports;   /* key id -> record */
std::unordered_map<void*, uint64_t> g_export_of;      /* allocation base -> key id */
uint64_t g_next_id = 1;                               /* never reused */

/* ---- the key blob (UCG_BUILTIN_DEV_IPC_HANDLE_BYTES, opaque to callers) --- */
struct ipc_blob {
    uint64_t magic;
    uint32_t kind;
    uint32_t pid;      /* exporter */
    uint64_t token;    /* exporter's key server (random per process) */
    uint64_t id;       /* key id at the exporter */
    uint64_t offset;   /* of the exported pointer in its allocation */
    uint64_t size;     /* of the allocation */
};
static_assert(sizeof(ipc_blob) <= UCG_BUILTIN_DEV_IPC_HANDLE_BYTES,
              "IPC blob does not fit the ABI size");
constexpr uint64_t kIpcMagic = 0x5543475f49504332ull;   /* "UCG_IPC2" */

/* key server protocol: request {id}, reply {status, kind, size, ih} plus the
 * allocation's fd (SCM_RIGHTS) for KIND_VMM */
struct key_request {
    uint64_t magic;
    uint64_t id;
};
struct key_reply {
    int32_t            status;      /* UCS_OK, or UCS_ERR_NO_RESOURCE: stale key */
    uint32_t           kind;
    uint64_t           size;
    hipIpcMemHandle_t  ih;
};

uint64_t g_token;           /* 0 until the server runs */
int      g_listen = -1;

std::string server_name(uint32_t pid, uint64_t token)
{
    char b[64];
    snprintf(b, sizeof(b), "xucg_ipc_%u_%016llx", pid, (unsigned long long)token);
    return b;
}

socklen_t abstract_addr(const std::string &name, sockaddr_un *a)
{
    memset(a, 0, sizeof(*a));
    a->sun_family = AF_UNIX;
    memcpy(a->sun_path + 1, name.data(), name.size());       /* abstract namespace */
    return (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + name.size());
}

bool read_full(int s, void *p, size_t n)
{
    char *c = static_cast<char*>(p);
    while (n) {
        const ssize_t r = read(s, c, n);
        if (r <= 0) {
            if (r < 0 && errno == EINTR) continue;
            return false;
        }
        c += r;
        n -= (size_t)r;
    }
    return true;
}

bool send_reply(int s, const key_reply &rep, int fd)
{
    iovec iov = {(void*)&rep, sizeof(rep)};
    msghdr mh = {};
    mh.msg_iov = &iov;
    mh.msg_iovlen = 1;
    char cbuf[CMSG_SPACE(sizeof(int))];
    if (fd >= 0) {
        memset(cbuf, 0, sizeof(cbuf));
        mh.msg_control = cbuf;
        mh.msg_controllen = sizeof(cbuf);
        cmsghdr *c = CMSG_FIRSTHDR(&mh);
        c->cmsg_level = SOL_SOCKET;
        c->cmsg_type = SCM_RIGHTS;
        c->cmsg_len = CMSG_LEN(sizeof(int));
        memcpy(CMSG_DATA(c), &fd, sizeof(int));
    }
    ssize_t r;
    do {
        r = sendmsg(s, &mh, MSG_NOSIGNAL);
    } while (r < 0 && errno == EINTR);
    return r == (ssize_t)sizeof(rep);
}

/* One request per connection. Only processes of this user are served. */
void serve_one(int s)
{
    key_request rq;
    key_reply rep;
    memset(&rep, 0, sizeof(rep));
    rep.status = UCS_ERR_INVALID_PARAM;
    int fd = -1;
    ucred cr;
    socklen_t cl = sizeof(cr);
    if (getsockopt(s, SOL_SOCKET, SO_PEERCRED, &cr, &cl) != 0 || cr.uid != getuid() ||
        !read_full(s, &rq, sizeof(rq)) || rq.magic != kIpcMagic) {
        send_reply(s, rep, -1);
        return;
    }
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_exports.find(rq.id);
        if (it == g_exports.end()) {
            rep.status = UCS_ERR_NO_RESOURCE;            /* retired: freed since */
        } else {
            const export_rec &e = it->second;
            rep.kind = (uint32_t)e.kind;
            rep.size = e.size;
            rep.status = UCS_OK;
            if (e.kind == KIND_VMM) {
                fd = dup(e.fd);
                if (fd < 0) rep.status = UCS_ERR_IO_ERROR;
            } else {
                /* the allocation at that address must still be the exported one */
                unsigned long long id = 0;
                const hipError_t he = hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID,
                                                             (hipDeviceptr_t)e.base);
                if (he != hipSuccess || id != e.buffer_id) {
                    rep.status = UCS_ERR_NO_RESOURCE;
                    (void)hipGetLastError();
                } else {
                    rep.ih = e.ih;
                }
            }
        }
    }
    send_reply(s, rep, rep.status == UCS_OK ? fd : -1);
    if (fd >= 0) {
        close(fd);
    }
}

void serve(int ls)
{
    for (;;) {
        const int s = accept4(ls, nullptr, nullptr, SOCK_CLOEXEC);
        if (s < 0) {
            if (errno == EINTR || errno == ECONNABORTED || errno == EMFILE ||
                errno == ENFILE || errno == ENOBUFS || errno == ENOMEM) {
                continue;
            }
            return;                                   /* the socket is gone */
        }
        serve_one(s);
        close(s);
    }
}

/* a forked child has no server thread: it starts its own on first export */
void after_fork_child()
{
    if (g_listen >= 0) {
        close(g_listen);
    }
    g_listen = -1;
    g_token = 0;
}

/* Start the key server once per process (first export). Caller holds g_mu. */
ucs_status_t server_start()
{
    static std::once_flag once;
    std::call_once(once, [] { pthread_atfork(nullptr, nullptr, after_fork_child); });
    if (g_listen >= 0) {
        return UCS_OK;
    }
    uint64_t tok = 0;
    const int r = open("/dev/urandom", O_RDONLY | O_CLOEXEC);
    if (r >= 0) {
        if (read(r, &tok, sizeof(tok)) != (ssize_t)sizeof(tok)) tok = 0;
        close(r);
    }
    tok ^= now_ns() ^ ((uint64_t)getpid() << 32);
    tok |= 1;
    const int ls = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (ls < 0) {
        return set_error(UCS_ERR_IO_ERROR, "ipc key server", strerror(errno));
    }
    sockaddr_un a;
    const socklen_t al = abstract_addr(server_name((uint32_t)getpid(), tok), &a);
    if (bind(ls, (sockaddr*)&a, al) != 0 || listen(ls, 128) != 0) {
        const int e = errno;
        close(ls);
        return set_error(UCS_ERR_IO_ERROR, "ipc key server", strerror(e));
    }
    std::thread(serve, ls).detach();
    g_listen = ls;
    g_token = tok;
    return UCS_OK;
}

/* Ask member (pid, token) for key `id`: the reply and, for KIND_VMM, the fd */
ucs_status_t fetch_key(const ipc_blob &b, key_reply *rep, int *fd)
{
    *fd = -1;
    const int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (s < 0) {
        return set_error(UCS_ERR_IO_ERROR, "ipc_import", strerror(errno));
    }
    sockaddr_un a;
    const socklen_t al = abstract_addr(server_name(b.pid, b.token), &a);
    int rc;
    do {
        rc = connect(s, (sockaddr*)&a, al);
    } while (rc != 0 && errno == EINTR);
    if (rc != 0) {
        const int e = errno;
        close(s);
        return set_error(UCS_ERR_NO_RESOURCE, "ipc_import",
                         (std::string("the exporter's key server is gone: ") + strerror(e)).c_str());
    }
    const key_request rq = {kIpcMagic, b.id};
    char cbuf[CMSG_SPACE(sizeof(int))];
    iovec iov = {rep, sizeof(*rep)};
    msghdr mh = {};
    mh.msg_iov = &iov;
    mh.msg_iovlen = 1;
    mh.msg_control = cbuf;
    mh.msg_controllen = sizeof(cbuf);
    ssize_t r = -1;
    if (write(s, &rq, sizeof(rq)) == (ssize_t)sizeof(rq)) {
        do {
            r = recvmsg(s, &mh, MSG_WAITALL | MSG_CMSG_CLOEXEC);
        } while (r < 0 && errno == EINTR);
    }
    close(s);
    if (r != (ssize_t)sizeof(*rep)) {
        return set_error(UCS_ERR_IO_ERROR, "ipc_import", "no reply from the key server");
    }
    for (cmsghdr *c = CMSG_FIRSTHDR(&mh); c; c = CMSG_NXTHDR(&mh, c)) {
        if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS) {
            memcpy(fd, CMSG_DATA(c), sizeof(int));
        }
    }
    if (rep->status != UCS_OK) {
        if (*fd >= 0) {
            close(*fd);
            *fd = -1;
        }
        return set_error((ucs_status_t)rep->status, "ipc_import",
                         rep->status == UCS_ERR_NO_RESOURCE
                             ? "stale key: the exported allocation was freed since"
                             : "the key server refused the key");
    }
    if (rep->kind == KIND_VMM && *fd < 0) {
        return set_error(UCS_ERR_IO_ERROR, "ipc_import", "no file descriptor in the reply");
    }
    return UCS_OK;
}

/* ---- imports (mapped once per key, reference counted) -------------------- */
struct import_rec {
    int      kind;      /* KIND_VMM, KIND_PLAIN, or 0: this process's own memory */
    char    *base;      /* the mapping (or the own allocation) */
    size_t   size;
    hipMemGenericAllocationHandle_t handle;   /* KIND_VMM */
    unsigned refs;
};
typedef std::tuple<uint32_t, uint64_t, uint64_t> import_key;   /* pid, token, id */
std::map<import_key, import_rec> g_imports;
std::unordered_multimap<void*, import_key> g_import_ptr;     /* pointer handed out -> key */

hipMemAccessDesc rw_access(int device)
{
    hipMemAccessDesc d;
    memset(&d, 0, sizeof(d));
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = device;
    d.flags = hipMemAccessFlagsProtReadWrite;
    return d;
}

/* How hipMemImportFromShareableHandle takes a POSIX fd: as the value cast
 * to a pointer (CUDA's convention; /opt/rocm 7.2's runtime) or as the address
 * of an int holding it (the ROCm 7.0 runtime PyTorch bundles dereferences
 * it: the value convention crashed there, r04c). Found once per process on an
 * allocation of its own (detect_fd_convention) and remembered. -1 unknown,
 * 0 value, 1 address. */
std::atomic<int> g_fd_convention{-1};

/* The int the address form points at. Its address's low 32 bits must be at
 * least 2^24, far above any fd number: of two addresses 16 MiB apart one
 * always is, so the box spans 16 MiB of untouched (unbacked) bss. */
int g_fd_box[((16u << 20) + 64) / sizeof(int)];
std::mutex g_fd_box_mu;

int *fd_box()
{
    int *p = g_fd_box;
    if ((uint32_t)(uintptr_t)p < (1u << 24)) {
        p += (16u << 20) / sizeof(int);
    }
    return p;
}

/* Find the convention once, on an allocation of this process's own: an
 * address-form import of an fd known to be good fails only on a value-form
 * runtime, and only then is the value form tried (on that same good fd). A
 * failing import of a peer's fd can then never send the value form to a
 * dereferencing runtime. Caller holds g_fd_box_mu. */
int detect_fd_convention(int device)
{
    const hipMemAllocationHandleType t = hipMemHandleTypePosixFileDescriptor;
    hipMemAllocationProp prop;
    memset(&prop, 0, sizeof(prop));
    prop.type = hipMemAllocationTypePinned;
    prop.requestedHandleType = t;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    hipMemGenericAllocationHandle_t own, imp;
    if (hipMemCreate(&own, kGran, &prop, 0) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    int fd = -1, conv = -1;
    if (hipMemExportToShareableHandle(&fd, own, t, 0) == hipSuccess && fd >= 0) {
        int *p = fd_box();
        *p = fd;
        if (hipMemImportFromShareableHandle(&imp, (void*)p, t) == hipSuccess) {
            conv = 1;
        } else {
            (void)hipGetLastError();
            if (hipMemImportFromShareableHandle(&imp, (void*)(intptr_t)fd, t) == hipSuccess) {
                conv = 0;
            }
        }
        if (conv >= 0) {
            (void)hipMemRelease(imp);
        }
        close(fd);
    }
    (void)hipGetLastError();
    (void)hipMemRelease(own);
    return conv;
}

hipError_t import_fd(hipMemGenericAllocationHandle_t *h, int fd, int device)
{
    const hipMemAllocationHandleType t = hipMemHandleTypePosixFileDescriptor;
    std::lock_guard<std::mutex> g(g_fd_box_mu);
    int conv = g_fd_convention.load(std::memory_order_relaxed);
    if (conv < 0) {
        conv = detect_fd_convention(device);
        if (conv < 0) {
            return hipErrorNotSupported;        /* no shareable memory here */
        }
        g_fd_convention.store(conv, std::memory_order_relaxed);
    }
    if (conv == 1) {
        int *p = fd_box();
        *p = fd;
        return hipMemImportFromShareableHandle(h, (void*)p, t);
    }
    return hipMemImportFromShareableHandle(h, (void*)(intptr_t)fd, t);
}

/* map an imported VMM allocation (fd) at a new reservation of this process */
ucs_status_t va_room(size_t bytes, const char *what);
void va_unclaim(size_t bytes);

ucs_status_t map_vmm(int fd, size_t size, int device, import_rec *m)
{
    const ucs_status_t room = va_room(size, "ipc_import");
    if (room != UCS_OK) {
        return room;
    }
    hipMemGenericAllocationHandle_t h;
    hipError_t e = import_fd(&h, fd, device);
    if (e != hipSuccess) {
        va_unclaim(size);
        return hip_status(e, "import_fd(&h, fd, device)");
    }
    void *va = nullptr;
    e = hipMemAddressReserve(&va, size, kGran, nullptr, 0);
    va_unclaim(size);
    if (e == hipSuccess) {
        e = hipMemMap(va, size, 0, h, 0);
        if (e == hipSuccess) {
            const hipMemAccessDesc d = rw_access(device);
            e = hipMemSetAccess(va, size, &d, 1);
            if (e != hipSuccess) {
                (void)hipMemUnmap(va, size);
            }
        }
        if (e != hipSuccess) {
            (void)hipMemAddressFree(va, size);
        }
    }
    if (e != hipSuccess) {
        (void)hipMemRelease(h);
        return hip_status(e, "ipc_import: map of the peer's allocation");
    }
    m->kind = KIND_VMM;
    m->base = static_cast<char*>(va);
    m->size = size;
    m->handle = h;
    return UCS_OK;
}

/* Address ranges of this shim's mappings are never given back (round 4). A
 * range mapped again to other physical memory was read through stale
 * translations: peers read the previous allocation's data, or zeros, through
 * a fresh mapping of a new allocation at an old address
 * (tools/va_reuse_probe). So an allocation or import, once
 * unmapped, leaves its reservation behind; physical memory goes back at once.
 * The retired ranges are counted (ucg_builtin_dev_mem_stats) and bounded
 * (round 5): past UCX_BUILTIN_DEV_VA_RETIRED_MAX (default
 * 64 TiB, half of the 128 TiB a process's GPU virtual address space spans)
 * a new shareable allocation or import fails with UCS_ERR_EXCEEDS_LIMIT
 * instead of running the address space out; half-way there a warning is
 * printed once. */
std::atomic<uint64_t> g_va_retired{0};
std::atomic<uint64_t> g_va_retired_ranges{0};
std::atomic<uint64_t> g_va_retired_max_set{0};        /* 0: the environment's */
std::atomic<bool>     g_va_warned{false};

uint64_t va_retired_max()
{
    const uint64_t set = g_va_retired_max_set.load(std::memory_order_relaxed);
    if (set) {
        return set;
    }
    static const uint64_t lim = parse_bytes(getenv("UCX_BUILTIN_DEV_VA_RETIRED_MAX"),
                                            (uint64_t)64 << 40);
    return lim;
}

/* may a new range of `bytes` be reserved? (UCS_ERR_EXCEEDS_LIMIT, named, if
 * the retired ranges are past the cap). The check and the claim are one
 * compare-and-swap on the retired count plus the claims in flight (ADVICE
 * r05: threads checking at once could together pass the cap); the caller
 * gives the claim back with va_unclaim once its range is mapped or failed -
 * the range counts again when it is retired. */
std::atomic<uint64_t> g_va_claimed{0};

ucs_status_t va_room(size_t bytes, const char *what)
{
    const uint64_t cap = va_retired_max();
    uint64_t c = g_va_claimed.load(std::memory_order_relaxed);
    for (;;) {
        const uint64_t r = g_va_retired.load(std::memory_order_relaxed);
        if (r + c + bytes > cap) {
            char b[220];
            snprintf(b, sizeof(b), "retired address ranges %llu B + %llu B in flight + %zu B "
                     "past UCX_BUILTIN_DEV_VA_RETIRED_MAX %llu B (never-remapped ranges, "
                     "DESIGN.md 6)", (unsigned long long)r, (unsigned long long)c, bytes,
                     (unsigned long long)cap);
            return set_error(UCS_ERR_EXCEEDS_LIMIT, what, b);
        }
        if (g_va_claimed.compare_exchange_weak(c, c + bytes)) {
            return UCS_OK;
        }
    }
}

void va_unclaim(size_t bytes)
{
    g_va_claimed.fetch_sub(bytes);
}

void va_retire(size_t bytes)
{
    const uint64_t r = g_va_retired.fetch_add(bytes) + bytes;
    g_va_retired_ranges++;
    if (r > va_retired_max() / 2 && !g_va_warned.exchange(true)) {
        fprintf(stderr, "xucg: %llu B of GPU virtual address space retired by unmapped "
                "shareable allocations and imports, past half of "
                "UCX_BUILTIN_DEV_VA_RETIRED_MAX (%llu B)\n", (unsigned long long)r,
                (unsigned long long)va_retired_max());
    }
}

void unmap_import(import_rec &m)
{
    if (m.kind == KIND_VMM) {
        (void)hipMemUnmap(m.base, m.size);
        (void)hipMemRelease(m.handle);
        va_retire(m.size);
    } else if (m.kind == KIND_PLAIN) {
        (void)hipIpcCloseMemHandle(m.base);
    }
}

}  // namespace

/* XUCG_NATIVE_BACKTRACE=1 (diagnostics, host code only): a SIGSEGV or
 * SIGBUS prints the native stack to stderr, then the previous handler (e.g.
 * Python's faulthandler) runs as before. Offsets into this library resolve
 * with addr2line against the same build. */
namespace {
struct sigaction g_prev_segv, g_prev_bus;

void native_backtrace(int sig, siginfo_t *si, void *uc)
{
    static const char hdr[] = "xucg: fatal signal, native stack:\n";
    (void)!write(2, hdr, sizeof(hdr) - 1);
    void *f[64];
    backtrace_symbols_fd(f, backtrace(f, 64), 2);
    const struct sigaction &prev = sig == SIGBUS ? g_prev_bus : g_prev_segv;
    sigaction(sig, &prev, nullptr);          /* the fault repeats into it */
    (void)si;
    (void)uc;
}

__attribute__((constructor)) void native_backtrace_init()
{
    const char *e = getenv("XUCG_NATIVE_BACKTRACE");
    if (e == nullptr || e[0] != '1') {
        return;
    }
    void *f[1];
    (void)backtrace(f, 1);                   /* load libgcc before any fault */
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = native_backtrace;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_prev_segv);
    sigaction(SIGBUS, &sa, &g_prev_bus);
}
}  // namespace

/* ---- peer mapping ---------------------------------------------------------- */
ucs_status_t ucg_builtin_dev_ipc_export(ucg_builtin_dev_ctx_t *ctx,
                                        const void *dev_ptr, void *handle)
{
    if (ctx == nullptr || dev_ptr == nullptr || handle == nullptr) {
        return set_error(UCS_ERR_INVALID_PARAM, "ipc_export", "bad arguments");
    }
    HIP_TRY(hipSetDevice(dev_ctx_device(ctx)));
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    HIP_TRY(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)dev_ptr));

    std::lock_guard<std::mutex> g(g_mu);
    ucs_status_t st = server_start();
    if (st != UCS_OK) {
        return st;
    }
    auto own = g_allocs.find((void*)base);
    uint64_t id = 0;
    auto ex = g_export_of.find((void*)base);
    if (ex != g_export_of.end()) {
        id = ex->second;
        export_rec &e = g_exports[id];
        if (e.kind == KIND_PLAIN) {
            /* caller memory: the allocation at this address may be a new one */
            unsigned long long bid = 0;
            if (hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, base) !=
                    hipSuccess || bid != e.buffer_id || e.size != size) {
                (void)hipGetLastError();
                g_exports.erase(id);               /* its keys are stale now */
                g_export_of.erase(ex);
                id = 0;
            }
        }
    }
    if (id == 0) {
        export_rec e;
        memset(&e, 0, sizeof(e));
        e.base = (void*)base;
        e.size = size;
        e.fd = -1;
        if (own != g_allocs.end() && own->second.kind == KIND_VMM) {
            e.kind = KIND_VMM;
            int fd = -1;
            HIP_TRY(hipMemExportToShareableHandle(&fd, own->second.handle,
                                                  hipMemHandleTypePosixFileDescriptor, 0));
            e.fd = fd;
        } else {
            e.kind = KIND_PLAIN;
            if (own != g_allocs.end() && !own->second.exported) {
                /* exported once, this allocation is kept for the life of the
                 * process (ucg_builtin_dev_free): within the keep cap */
                const uint64_t cap = keep_max(own->second.device);
                if (g_kept + own->second.bytes > cap) {
                    char b[220];
                    snprintf(b, sizeof(b), "memory kept for exported allocations %llu B + "
                             "%zu B past UCX_BUILTIN_DEV_KEEP_MAX %llu B (exported memory "
                             "is never given back, DESIGN.md 7)", (unsigned long long)g_kept,
                             own->second.bytes, (unsigned long long)cap);
                    return set_error(UCS_ERR_EXCEEDS_LIMIT, "ipc_export", b);
                }
            }
            HIP_TRY(hipPointerGetAttribute(&e.buffer_id, HIP_POINTER_ATTRIBUTE_BUFFER_ID,
                                           base));
            HIP_TRY(hipIpcGetMemHandle(&e.ih, (void*)base));
        }
        id = g_next_id++;
        g_exports[id] = e;
        g_export_of[(void*)base] = id;
        if (own != g_allocs.end()) {
            own->second.key_id = id;
            if (own->second.kind == KIND_PLAIN && !own->second.exported) {
                g_kept += own->second.bytes;
                const uint64_t cap = keep_max(own->second.device);
                if (g_kept > cap / 2 && !g_keep_warned) {
                    g_keep_warned = true;
                    fprintf(stderr, "xucg: %llu B kept for exported allocations (never "
                            "given back), past half of UCX_BUILTIN_DEV_KEEP_MAX (%llu B)\n",
                            (unsigned long long)g_kept, (unsigned long long)cap);
                }
            }
            own->second.exported = true;
        }
    }
    note_event('X', (void*)dev_ptr, (void*)base, size, 0);
    const export_rec &e = g_exports[id];
    ipc_blob b;
    memset(&b, 0, sizeof(b));
    b.magic  = kIpcMagic;
    b.kind   = (uint32_t)e.kind;
    b.pid    = (uint32_t)getpid();
    b.token  = g_token;
    b.id     = id;
    b.offset = (uint64_t)((const char*)dev_ptr - (const char*)base);
    b.size   = (uint64_t)size;
    memset(handle, 0, UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
    memcpy(handle, &b, sizeof(b));
    return UCS_OK;
}

ucs_status_t ucg_builtin_dev_ipc_import(ucg_builtin_dev_ctx_t *ctx,
                                        const void *handle, void **dev_ptr)
{
    if (ctx == nullptr || handle == nullptr || dev_ptr == nullptr) {
        return set_error(UCS_ERR_INVALID_PARAM, "ipc_import", "bad arguments");
    }
    ipc_blob b;
    memcpy(&b, handle, sizeof(b));
    if (b.magic != kIpcMagic || b.offset >= b.size ||
        (b.kind != KIND_VMM && b.kind != KIND_PLAIN)) {
        return set_error(UCS_ERR_INVALID_PARAM, "ipc_import", "not an exported handle");
    }
    const int device = dev_ctx_device(ctx);
    HIP_TRY(hipSetDevice(device));
    const import_key k{b.pid, b.token, b.id};
    const bool self = b.pid == (uint32_t)getpid() && b.token == g_token;
    if (self) {
        /* this process's own allocation: no mapping, but the key must still
         * be live */
        std::lock_guard<std::mutex> g(g_mu);
        auto ex = g_exports.find(b.id);
        if (ex == g_exports.end()) {
            note_event('S', nullptr, nullptr, (size_t)b.size, 0);
            return set_error(UCS_ERR_NO_RESOURCE, "ipc_import",
                             "stale key: the exported allocation was freed since");
        }
        auto it = g_imports.find(k);
        if (it != g_imports.end()) {
            it->second.refs++;
        } else {
            g_imports[k] = import_rec{0, static_cast<char*>(ex->second.base),
                                      ex->second.size, {}, 1};
        }
        *dev_ptr = static_cast<char*>(ex->second.base) + b.offset;
        g_import_ptr.emplace(*dev_ptr, k);
        return UCS_OK;
    }
    /* every import asks the exporter, so a retired key is refused even while
     * an earlier import of it is still held here (which keeps its mapping) */
    key_reply rep;
    int fd = -1;
    ucs_status_t st = fetch_key(b, &rep, &fd);
    if (st != UCS_OK) {
        std::lock_guard<std::mutex> g(g_mu);
        note_event('S', nullptr, nullptr, (size_t)b.size, (int)st);
        return st;
    }
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_imports.find(k);
        if (it != g_imports.end()) {
            if (fd >= 0) close(fd);
            it->second.refs++;
            *dev_ptr = it->second.base + b.offset;
            g_import_ptr.emplace(*dev_ptr, k);
            return UCS_OK;
        }
    }
    if (rep.size != b.size || rep.kind != b.kind) {
        if (fd >= 0) close(fd);
        return set_error(UCS_ERR_INVALID_PARAM, "ipc_import",
                         "the key server describes another allocation");
    }
    import_rec m;
    memset(&m, 0, sizeof(m));
    if (b.kind == KIND_VMM) {
        st = map_vmm(fd, (size_t)b.size, device, &m);
        close(fd);
        if (st != UCS_OK) {
            return st;
        }
    } else {
        void *base = nullptr;
        HIP_TRY(hipIpcOpenMemHandle(&base, rep.ih, hipIpcMemLazyEnablePeerAccess));
        /* the mapping must span the exporter's allocation; where the runtime
         * cannot answer the range query for an imported pointer, it must at
         * least know the pointer as device memory */
        hipDeviceptr_t mb = nullptr;
        size_t ms = 0;
        bool ok;
        if (hipMemGetAddressRange(&mb, &ms, (hipDeviceptr_t)base) == hipSuccess) {
            ok = mb == (hipDeviceptr_t)base && ms >= b.size;
        } else {
            (void)hipGetLastError();
            hipPointerAttribute_t at;
            memset(&at, 0, sizeof(at));
            ok = hipPointerGetAttributes(&at, base) == hipSuccess &&
                 at.type == hipMemoryTypeDevice;
            (void)hipGetLastError();
        }
        if (!ok) {
            (void)hipIpcCloseMemHandle(base);
            return set_error(UCS_ERR_INVALID_PARAM, "ipc_import",
                             "mapped range does not cover the exported allocation");
        }
        m.kind = KIND_PLAIN;
        m.base = static_cast<char*>(base);
        m.size = (size_t)b.size;
    }
    m.refs = 1;
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_imports.find(k);
    if (it != g_imports.end()) {
        /* another thread mapped it meanwhile: keep that one */
        unmap_import(m);
        it->second.refs++;
        *dev_ptr = it->second.base + b.offset;
    } else {
        g_imports[k] = m;
        *dev_ptr = m.base + b.offset;
    }
    g_import_ptr.emplace(*dev_ptr, k);
    note_event('I', *dev_ptr, g_imports[k].base, (size_t)b.size, 0);
    return UCS_OK;
}

ucs_status_t ucg_builtin_dev_ipc_release(ucg_builtin_dev_ctx_t *ctx, void *dev_ptr)
{
    if (ctx == nullptr || dev_ptr == nullptr) {
        return set_error(UCS_ERR_INVALID_PARAM, "ipc_release", "bad arguments");
    }
    import_rec m;
    bool last = false;
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto p = g_import_ptr.find(dev_ptr);
        if (p == g_import_ptr.end()) {
            return set_error(UCS_ERR_INVALID_PARAM, "ipc_release", "not an imported pointer");
        }
        const import_key k = p->second;
        g_import_ptr.erase(p);
        auto it = g_imports.find(k);
        if (it != g_imports.end() && --it->second.refs == 0) {
            m = it->second;
            last = true;
            g_imports.erase(it);
        }
    }
    if (last && m.kind) {
        /* nothing of this shim may still read it: the streams of this
         * device's contexts are drained, not the whole device (outside the
         * lock: the key server keeps answering peers meanwhile) */
        const hipError_t e = dev_streams_drain(dev_ctx_device(ctx));
        unmap_import(m);
        std::lock_guard<std::mutex> g(g_mu);
        note_event('C', dev_ptr, m.base, m.size, (int)e);
    }
    return UCS_OK;
}

/* ---- memory helpers -------------------------------------------------------- */
void *ucg_builtin_dev_malloc(ucg_builtin_dev_ctx_t *ctx, size_t bytes)
{
    void *p = nullptr;
    if (ctx) {
        (void)hipSetDevice(dev_ctx_device(ctx));
    }
    int device = 0;
    (void)hipGetDevice(&device);
    /* whole 2 MiB granules: a small hipMalloc may be carved out of a block
     * the runtime shares with other allocations, and such memory cannot be
     * exported through hipIpcGetMemHandle (ucg_builtin_dev_ipc_export) */
    bytes = round_gran(bytes);
    {
        std::lock_guard<std::mutex> g(g_mu);
        /* the most recently freed one of its size (equal keys keep their
         * insertion order) */
        auto c = g_plain_cache.upper_bound({device, bytes});
        if (c != g_plain_cache.begin() &&
            (c = std::prev(c))->first == std::make_pair(device, bytes)) {
            p = c->second.first;
            const bool was_exported = c->second.second;
            g_plain_cache.erase(c);
            (was_exported ? g_cached_exported : g_plain_cached) -= bytes;
            g_allocs[p] = own_alloc{KIND_PLAIN, device, bytes, {}, 0, was_exported, bytes};
            note_event('R', p, p, bytes, 0);
            return p;
        }
        /* else the smallest ever-exported one up to twice the size: those are
         * never given back, so a caller whose sizes vary reuses them rather
         * than adding one per size; what it holds beyond the request is
         * counted as slack (ucg_builtin_dev_mem_stats [10]) */
        for (auto x = g_plain_cache.lower_bound({device, bytes});
             x != g_plain_cache.end() && x->first.first == device &&
             x->first.second <= 2 * bytes; ++x) {
            if (x->second.second) {
                const size_t have = x->first.second;
                p = x->second.first;
                g_plain_cache.erase(x);
                g_cached_exported -= have;
                g_slack += have - bytes;
                g_allocs[p] = own_alloc{KIND_PLAIN, device, have, {}, 0, true, bytes};
                note_event('R', p, p, have, 0);
                return p;
            }
        }
    }
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipErrorOutOfMemory && plain_cache_drain(device) > 0) {
        /* the reuse cache held memory of other sizes: given back, once more,
         * on this allocation's device (the drain leaves it current) */
        (void)hipGetLastError();
        e = hipMalloc(&p, bytes);
    }
    if (e != hipSuccess) {
        hip_status(e, "hipMalloc");
        return nullptr;
    }
    std::lock_guard<std::mutex> g(g_mu);
    g_allocs[p] = own_alloc{KIND_PLAIN, device, bytes, {}, 0, false, bytes};
    note_event('M', p, p, bytes, 0);
    return p;
}

void *ucg_builtin_dev_malloc_shareable(ucg_builtin_dev_ctx_t *ctx, size_t bytes)
{
    /* UCX_BUILTIN_DEV_SHAREABLE=n: plain hipMalloc memory (hipIpc keys) where
     * peers cannot map each other's virtual-memory allocations; read at every
     * call, so a process can switch after probing (bench.py) */
    const char *knob = getenv("UCX_BUILTIN_DEV_SHAREABLE");
    if (knob && (knob[0] == 'n' || knob[0] == '0')) {
        return ucg_builtin_dev_malloc(ctx, bytes);
    }
    int device = 0;
    if (ctx) {
        device = dev_ctx_device(ctx);
        (void)hipSetDevice(device);
    } else {
        (void)hipGetDevice(&device);
    }
    bytes = round_gran(bytes);
    if (va_room(bytes, "malloc_shareable") != UCS_OK) {
        return nullptr;
    }
    hipMemAllocationProp prop;
    memset(&prop, 0, sizeof(prop));
    prop.type = hipMemAllocationTypePinned;
    prop.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    hipMemGenericAllocationHandle_t h;
    hipError_t e = hipMemCreate(&h, bytes, &prop, 0);
    if (e != hipSuccess) {
        va_unclaim(bytes);
        hip_status(e, "hipMemCreate");
        return nullptr;
    }
    void *va = nullptr;
    e = hipMemAddressReserve(&va, bytes, kGran, nullptr, 0);
    va_unclaim(bytes);
    if (e == hipSuccess) {
        e = hipMemMap(va, bytes, 0, h, 0);
        if (e == hipSuccess) {
            const hipMemAccessDesc d = rw_access(device);
            e = hipMemSetAccess(va, bytes, &d, 1);
            if (e != hipSuccess) {
                (void)hipMemUnmap(va, bytes);
            }
        }
        if (e != hipSuccess) {
            (void)hipMemAddressFree(va, bytes);
        }
    }
    if (e != hipSuccess) {
        (void)hipMemRelease(h);
        hip_status(e, "shareable allocation (reserve / map / access)");
        return nullptr;
    }
    std::lock_guard<std::mutex> g(g_mu);
    g_allocs[va] = own_alloc{KIND_VMM, device, bytes, h, 0, false, bytes};
    note_event('V', va, va, bytes, 0);
    return va;
}

int ucg_builtin_dev_is_shareable(const void *ptr)
{
    std::lock_guard<std::mutex> g(g_mu);
    for (const auto &kv : g_allocs) {
        const char *b = static_cast<const char*>(kv.first);
        if (kv.second.kind == KIND_VMM && (const char*)ptr >= b && (const char*)ptr < b + kv.second.bytes) {
            return 1;
        }
    }
    return 0;
}

void ucg_builtin_dev_free(ucg_builtin_dev_ctx_t *ctx, void *ptr)
{
    if (ptr == nullptr) {
        return;
    }
    own_alloc a;
    bool own = false;
    int fd = -1;
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_allocs.find(ptr);
        if (it != g_allocs.end()) {
            a = it->second;
            own = true;
            g_slack -= a.bytes - a.want;
            g_allocs.erase(it);
        }
        /* retire its key: a peer's import of it is refused from now on */
        auto ex = g_export_of.find(ptr);
        if (ex != g_export_of.end()) {
            fd = g_exports[ex->second].fd;
            g_exports.erase(ex->second);
            g_export_of.erase(ex);
        }
    }
    if (fd >= 0) {
        close(fd);
    }
    if (ctx) {
        (void)hipSetDevice(dev_ctx_device(ctx));
    }
    hipError_t e;
    if (own && a.kind == KIND_VMM) {
        /* nothing this shim queued may still use it (its contexts' streams
         * on the device, not the whole device: round 6). Peers that mapped
         * it keep the physical memory until they release their mapping. */
        e = dev_streams_drain(a.device);
        (void)hipMemUnmap(ptr, a.bytes);
        (void)hipMemRelease(a.handle);
        va_retire(a.bytes);                /* the range is never reused */
    } else if (own && a.kind == KIND_PLAIN) {
        /* as hipFree does: nothing queued may still use it; then kept for
         * the next allocation of its size (g_plain_cache), exported or not.
         * An allocation that was ever exported must not go back to the
         * runtime, so it is kept whatever the bound: the next hipMalloc
         * hands its address out again with other memory, and peers' fresh
         * hipIpcOpenMemHandle of a recycled address read another process's
         * buffer in 3,608 of 6,974 checks (12 processes,
         * tools/va_reuse_probe ipc). Reused here it is the same
         * memory. A buffer that a peer may still be reading is parked
         * instead (ucg_builtin_dev_park: ADVICE r04). Before it is handed
         * out again, the work this shim queued on it has drained: the
         * streams of the device's contexts (round 6: no device-wide sync,
         * which waited for RCCL's and the application's streams too). Only
         * never-exported bytes count against UCX_BUILTIN_DEV_CACHE_BYTES
         * (ADVICE r05); exported ones are bounded by the keep cap. */
        e = dev_streams_drain(a.device);
        bool kept = false;
        {
            std::lock_guard<std::mutex> g(g_mu);
            if (a.exported || g_plain_cached + a.bytes <= plain_cache_limit()) {
                g_plain_cache.emplace(std::make_pair(a.device, a.bytes),
                                      std::make_pair(ptr, a.exported));
                (a.exported ? g_cached_exported : g_plain_cached) += a.bytes;
                kept = true;
            }
        }
        if (!kept) {
            e = hipFree(ptr);
        }
    } else {
        e = hipFree(ptr);
    }
    std::lock_guard<std::mutex> g(g_mu);
    note_event('F', ptr, ptr, own ? a.bytes : 0, (int)e);
}

void ucg_builtin_dev_park(ucg_builtin_dev_ctx_t *ctx, void *ptr)
{
    if (ptr == nullptr) {
        return;
    }
    (void)ctx;
    int fd = -1;
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_allocs.find(ptr);
    if (it == g_allocs.end()) {
        return;                                  /* not this shim's: left alone */
    }
    g_parked += it->second.bytes;
    if (!(it->second.kind == KIND_PLAIN && it->second.exported)) {
        g_kept += it->second.bytes;              /* exported ones count already */
    }
    g_slack -= it->second.bytes - it->second.want;
    g_allocs.erase(it);                          /* never freed, never handed out */
    auto ex = g_export_of.find(ptr);
    if (ex != g_export_of.end()) {               /* its keys retire all the same */
        fd = g_exports[ex->second].fd;
        g_exports.erase(ex->second);
        g_export_of.erase(ex);
    }
    if (fd >= 0) {
        close(fd);
    }
    note_event('P', ptr, ptr, 0, 0);
}

void ucg_builtin_dev_mem_stats(uint64_t out[UCG_BUILTIN_DEV_NMEMSTATS])
{
    if (out == nullptr) {
        return;
    }
    std::lock_guard<std::mutex> g(g_mu);
    uint64_t live_vmm = 0, live_imp = 0;
    for (const auto &kv : g_allocs) {
        if (kv.second.kind == KIND_VMM) {
            live_vmm += kv.second.bytes;
        }
    }
    for (const auto &kv : g_imports) {
        if (kv.second.kind == KIND_VMM) {
            live_imp += kv.second.size;
        }
    }
    out[0] = g_va_retired.load();
    out[1] = g_va_retired_ranges.load();
    out[2] = va_retired_max();
    int device = 0;
    (void)hipGetDevice(&device);
    out[3] = g_plain_cached + g_cached_exported;
    out[4] = live_vmm;
    out[5] = live_imp;
    out[6] = g_parked;
    out[7] = g_kept;
    out[8] = keep_max(device);
    out[9] = g_cached_exported;
    out[10] = g_slack;
}

void ucg_builtin_dev_set_va_retired_max(uint64_t bytes)
{
    g_va_retired_max_set.store(bytes);
    g_va_warned.store(false);
}

void ucg_builtin_dev_set_keep_max(uint64_t bytes)
{
    g_keep_max_set.store(bytes);
    std::lock_guard<std::mutex> g(g_mu);
    g_keep_warned = false;
}

/* torch.cuda.memory.CUDAPluggableAllocator entry points: every tensor of a
 * process that installs them is a shareable allocation, so any tensor can be
 * exported by its physical allocation (xucg_amd.use_shareable_torch_memory) */
void *ucg_builtin_dev_torch_alloc(size_t bytes, int device, void *stream)
{
    (void)stream;
    (void)hipSetDevice(device);
    return ucg_builtin_dev_malloc_shareable(nullptr, bytes ? bytes : 1);
}

void ucg_builtin_dev_torch_free(void *ptr, size_t bytes, int device, void *stream)
{
    (void)bytes;
    (void)stream;
    (void)hipSetDevice(device);
    ucg_builtin_dev_free(nullptr, ptr);        /* drains the shim's streams first */
}

/* Diagnostics for a buffer found corrupted (tests/_worker_topo.py): what the
 * runtime says about the address now, whether it lies in a live allocation or
 * an import of this shim, and the recorded memory events whose range comes
 * within 4 MiB of it, oldest first. */
size_t ucg_builtin_dev_debug_ptr(ucg_builtin_dev_ctx_t *ctx, const void *ptr, char *out,
                                 size_t max)
{
    std::string t;
    char line[256];
    if (ctx) {
        (void)hipSetDevice(dev_ctx_device(ctx));
    }
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    const hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr);
    snprintf(line, sizeof(line), "address %p: runtime range %s base %p size %zu\n", ptr,
             e == hipSuccess ? "ok" : hipGetErrorString(e), (void*)base, size);
    t += line;
    (void)hipGetLastError();
    hipPointerAttribute_t at;
    memset(&at, 0, sizeof(at));
    const hipError_t ea = hipPointerGetAttributes(&at, ptr);
    snprintf(line, sizeof(line), "attributes %s: type %d device %d devptr %p\n",
             ea == hipSuccess ? "ok" : hipGetErrorString(ea), (int)at.type, at.device,
             at.devicePointer);
    t += line;
    (void)hipGetLastError();
    const uintptr_t a = (uintptr_t)ptr, win = (uintptr_t)4 << 20;
    std::lock_guard<std::mutex> g(g_mu);
    for (const auto &kv : g_allocs) {
        const uintptr_t p = (uintptr_t)kv.first;
        if (a >= p && a < p + kv.second.bytes) {
            snprintf(line, sizeof(line), "own allocation %p + %zu %s key %llu\n", kv.first,
                     kv.second.bytes, kv.second.kind == KIND_VMM ? "shareable" : "plain",
                     (unsigned long long)kv.second.key_id);
            t += line;
        }
    }
    for (const auto &kv : g_imports) {
        const uintptr_t p = (uintptr_t)kv.second.base;
        if (a >= p && a < p + kv.second.size) {
            snprintf(line, sizeof(line), "import of pid %u key %llu mapped at %p + %zu (%s)\n",
                     std::get<0>(kv.first), (unsigned long long)std::get<2>(kv.first),
                     (void*)kv.second.base, kv.second.size,
                     kv.second.kind == KIND_VMM ? "shareable" :
                     kv.second.kind == KIND_PLAIN ? "hipIpc" : "own");
            t += line;
        }
    }
    const uint64_t first = g_nevents > kMemEvents ? g_nevents - kMemEvents : 0;
    const uint64_t now = now_ns();
    for (uint64_t i = first; i < g_nevents; i++) {
        const mem_event &ev = g_events[i % kMemEvents];
        const uintptr_t lo = (uintptr_t)(ev.base ? ev.base : ev.ptr);
        if (lo + win > a && lo < a + win) {
            snprintf(line, sizeof(line), "event #%llu %c ptr %p base %p bytes %zu rc %d, %.3f ms ago\n",
                     (unsigned long long)i, ev.kind, ev.ptr, ev.base, ev.bytes, ev.rc,
                     (double)(now - ev.ns) * 1e-6);
            t += line;
        }
    }
    if (out && max) {
        const size_t n = t.size() < max - 1 ? t.size() : max - 1;
        memcpy(out, t.data(), n);
        out[n] = '\0';
    }
    return t.size();
}
