/*
 * builtin_shm.c - f2: a minimal shared-memory active-message transport for the
 * builtin engine (include/ucg_builtin_ops.h): per-pair SPSC rings of AM-short
 * cells (UCS_ERR_NO_RESOURCE when full, as uct_ep_am_short), delivery with
 * the data borrowed for the callback only, the incast cell of the UCX
 * collectives extension, and a barrier for set-up and tear-down.
 */
#define _GNU_SOURCE
#include "builtin_int.h"

#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

static ring_ctl_t *ring_ctl(ucg_builtin_shm_iface_t *it, unsigned src, unsigned dst)
{
    return (ring_ctl_t*)(it->seg + it->ctl_bytes +
                         ((size_t)src * it->members + dst) * it->ring_bytes);
}

static cell_t *ring_cell(ucg_builtin_shm_iface_t *it, ring_ctl_t *r, uint64_t idx)
{
    return (cell_t*)((char*)r + sizeof(ring_ctl_t) + (idx % it->cells) * it->cell_size);
}

static incast_ctl_t *incast_ctl(ucg_builtin_shm_iface_t *it, unsigned member)
{
    return (incast_ctl_t*)(it->seg + it->incast_base + member * it->incast_bytes);
}

static incast_cell_t *incast_cell(ucg_builtin_shm_iface_t *it, unsigned member,
                                  unsigned idx)
{
    return (incast_cell_t*)((char*)incast_ctl(it, member) + sizeof(incast_ctl_t) +
                            (size_t)idx * it->incast_cell_size);
}

/* The object's header (the first SEG_HDR_BYTES): the barrier counter at 0,
 * then who made it. Member 0 creates the object (O_EXCL) and stamps it with
 * its pid, its pid namespace, the job's token and a random instance; the
 * others map it once it is stamped by a live creator of their own job and the
 * name still refers to that instance. An object left behind by a dead
 * creator (a crashed job) is unlinked and made anew; one whose creator is
 * alive belongs to another job with the same name and is refused
 * (UCS_ERR_BUSY: set a job uid) - by member 0, and (round 5) by
 * every other member too when both jobs carry a token (job_token). A creator
 * in another pid namespace (containers sharing /dev/shm) cannot be probed
 * with kill(): its object is taken as live, and recycled by member 0 only
 * when it carries this job's own token. Closing marks the object closed
 * before the last barrier, so a member that reopens the name at once waits
 * for the next instance. ADVICE r03: two jobs without a job uid, or a new job
 * over a crashed one's object, shared rings and the barrier counter. */
typedef struct {
    _Atomic uint64_t arrive;            /* ucg_builtin_shm_barrier */
    uint64_t         pad[7];
    _Atomic uint64_t stamp;             /* SHM_STAMP once set up, SHM_CLOSED at close */
    uint64_t         owner;             /* the creator's pid */
    uint64_t         instance;          /* random, per creation */
    uint64_t         seg_bytes;
    uint64_t         members;
    uint64_t         pidns;             /* the creator's pid namespace (0: unknown) */
    uint64_t         job;               /* the creator's job token (0: none) */
} seg_hdr_t;
_Static_assert(sizeof(seg_hdr_t) <= SEG_HDR_BYTES, "segment header size");
#define SHM_STAMP  0x58554347534d3031ull         /* "XUCGSM01" */
#define SHM_CLOSED 0x58554347534d4344ull

static member_ctl_t *member_ctl(ucg_builtin_shm_iface_t *it, unsigned member)
{
    return (member_ctl_t*)(it->seg + SEG_HDR_BYTES) + member;
}

/* a process that exited but was not reaped yet (a zombie: its launcher has
 * not waited for it) is gone too, though kill() still finds it */
static int pid_zombie(uint64_t pid)
{
    char path[64], buf[256], *p;
    ssize_t n;
    int fd;
    snprintf(path, sizeof(path), "/proc/%llu/stat", (unsigned long long)pid);
    if ((fd = open(path, O_RDONLY | O_CLOEXEC)) < 0) {
        return 0;
    }
    n = read(fd, buf, sizeof(buf) - 1);
    close(fd);
    if (n <= 0) {
        return 0;
    }
    buf[n] = 0;
    /* "pid (comm) S ...": the state follows the last ')' */
    p = strrchr(buf, ')');
    return p && p[1] == ' ' && (p[2] == 'Z' || p[2] == 'X');
}

static int pid_alive(uint64_t pid)
{
    return pid != 0 && (kill((pid_t)pid, 0) == 0 || errno != ESRCH) && !pid_zombie(pid);
}

/* this process's pid namespace: the inode of /proc/self/ns/pid (0: unknown) */
static uint64_t pid_ns(void)
{
    struct stat sb;
    return stat("/proc/self/ns/pid", &sb) == 0 ? (uint64_t)sb.st_ino : 0;
}

/* the creator `pid` of namespace `ns`: 1 alive, 0 gone, -1 cannot tell (a
 * pid of another namespace means nothing to kill() here) */
static int owner_state(uint64_t pid, uint64_t ns)
{
    const uint64_t mine = pid_ns();
    if (ns != 0 && mine != 0 && ns != mine) {
        return -1;
    }
    return pid_alive(pid);
}

/* This job's token, the same in every member of one launch: FNV-1a of
 * UCX_BUILTIN_JOB_TOKEN, else of the launcher's job id (PMIx namespace, Open
 * MPI's job id, Slurm's job.step, torchrun's run id, the rendezvous
 * MASTER_ADDR:MASTER_PORT); 0 when there is none (a peer can then not tell
 * another job's object from its own: set a job uid). Exported for the tests
 * as ucg_builtin_shm_job_token. */
static uint64_t job_token(void)
{
    static const char *vars[][2] = {{"UCX_BUILTIN_JOB_TOKEN", NULL},
                                    {"PMIX_NAMESPACE", NULL},
                                    {"OMPI_MCA_ess_base_jobid", NULL},
                                    {"SLURM_JOB_ID", "SLURM_STEP_ID"},
                                    {"TORCHELASTIC_RUN_ID", NULL},
                                    {"MASTER_ADDR", "MASTER_PORT"}};
    unsigned i;
    for (i = 0; i < sizeof(vars) / sizeof(vars[0]); i++) {
        const char *a = getenv(vars[i][0]), *b = vars[i][1] ? getenv(vars[i][1]) : "";
        const char *parts[3];
        uint64_t h = 0xcbf29ce484222325ull;
        unsigned k;
        /* torchrun sets TORCHELASTIC_RUN_ID=none for every static-rendezvous
         * job without --rdzv-id: no job's id, the rendezvous
         * address decides */
        if (a == NULL || *a == 0 || b == NULL || strcmp(a, "none") == 0) {
            continue;
        }
        parts[0] = a;
        parts[1] = *b ? ":" : "";
        parts[2] = b;
        for (k = 0; k < 3; k++) {
            const unsigned char *c;
            for (c = (const unsigned char*)parts[k]; *c; c++) {
                h = (h ^ *c) * 0x100000001b3ull;
            }
        }
        return h ? h : 1;
    }
    return 0;
}

uint64_t ucg_builtin_shm_job_token(void)
{
    return job_token();
}

/* this member is attached: its process, for the others' liveness probes */
static void member_attach(ucg_builtin_shm_iface_t *it)
{
    member_ctl_t *m = member_ctl(it, it->my);
    m->pidns = pid_ns();
    atomic_store_explicit(&m->pid, (uint64_t)getpid(), memory_order_release);
}

/* the first failure sticks: later ones (a timeout after a reset) keep it */
static ucs_status_t set_broken(ucg_builtin_shm_iface_t *it, ucs_status_t st)
{
    int ok = UCS_OK;
    atomic_compare_exchange_strong_explicit(&it->broken, &ok, (int)st, memory_order_acq_rel,
                                            memory_order_acquire);
    return (ucs_status_t)atomic_load_explicit(&it->broken, memory_order_acquire);
}

static inline ucs_status_t broken_status(ucg_builtin_shm_iface_t *it)
{
    return (ucs_status_t)atomic_load_explicit(&it->broken, memory_order_acquire);
}

UCG_INTERNAL int shm_peer_check(ucg_builtin_shm_iface_t *it)
{
    const uint64_t t = (uint64_t)(now_s() * 1e9);
    uint64_t last = atomic_load_explicit(&it->live_check_ns, memory_order_relaxed);
    int dead = atomic_load_explicit(&it->dead, memory_order_acquire);
    unsigned m;
    /* one prober per interval: the owner and the timer threads race for it */
    if (dead || t - last < (uint64_t)(PEER_CHECK_S * 1e9) ||
        !atomic_compare_exchange_strong_explicit(&it->live_check_ns, &last, t,
                                                 memory_order_relaxed,
                                                 memory_order_relaxed)) {
        return atomic_load_explicit(&it->dead, memory_order_acquire) - 1;
    }
    for (m = 0; m < it->members; m++) {
        const member_ctl_t *mc = member_ctl(it, m);
        const uint64_t pid = atomic_load_explicit(&mc->pid, memory_order_acquire);
        int none = 0;
        /* not attached yet, or in another pid namespace: cannot tell */
        if (m == it->my || pid == 0 || owner_state(pid, mc->pidns) != 0) {
            continue;
        }
        if (atomic_compare_exchange_strong_explicit(&it->dead, &none, (int)m + 1,
                                                    memory_order_acq_rel,
                                                    memory_order_acquire)) {
            fprintf(stderr, "ucg_builtin_shm(%s): member %u (pid %llu) is gone\n", it->name,
                    m, (unsigned long long)pid);
        }
        set_broken(it, UCS_ERR_CONNECTION_RESET);
        return atomic_load_explicit(&it->dead, memory_order_acquire) - 1;
    }
    return -1;
}

UCG_INTERNAL void shm_abandon(ucg_builtin_shm_iface_t *it, unsigned slot, uint64_t word)
{
    atomic_store_explicit(&member_ctl(it, it->my)->abandoned[slot % UNEXP_GROUPS], word,
                          memory_order_release);
}

UCG_INTERNAL uint64_t shm_abandoned(ucg_builtin_shm_iface_t *it, unsigned member,
                                    unsigned slot)
{
    return atomic_load_explicit(&member_ctl(it, member)->abandoned[slot % UNEXP_GROUPS],
                                memory_order_acquire);
}

/* an object of another job: both sides carry a token and they differ */
static int foreign_job(uint64_t job)
{
    const uint64_t mine = job_token();
    return job != 0 && mine != 0 && job != mine;
}

/* the header of the object the name refers to now (zeros if none) */
static void peek_hdr(const char *name, seg_hdr_t *out)
{
    struct stat sb;
    seg_hdr_t *h;
    int fd = shm_open(name, O_RDONLY, 0);
    memset(out, 0, sizeof(*out));
    if (fd < 0) {
        return;
    }
    if (fstat(fd, &sb) == 0 && (size_t)sb.st_size >= sizeof(seg_hdr_t)) {
        h = mmap(NULL, sizeof(seg_hdr_t), PROT_READ, MAP_SHARED, fd, 0);
        if (h != MAP_FAILED) {
            out->stamp     = atomic_load_explicit(&h->stamp, memory_order_acquire);
            out->owner     = h->owner;
            out->instance  = h->instance;
            out->seg_bytes = h->seg_bytes;
            out->members   = h->members;
            out->pidns     = h->pidns;
            out->job       = h->job;
            munmap(h, sizeof(seg_hdr_t));
        }
    }
    close(fd);
}

static uint64_t random_u64(void)
{
    uint64_t v = 0;
    int fd = open("/dev/urandom", O_RDONLY | O_CLOEXEC);
    if (fd >= 0) {
        if (read(fd, &v, sizeof(v)) != (ssize_t)sizeof(v)) {
            v = 0;
        }
        close(fd);
    }
    return (v ^ (uint64_t)(now_s() * 1e9) ^ ((uint64_t)getpid() << 40)) | 1;
}

/* member 0: a new object under the name */
static int iface_create(ucg_builtin_shm_iface_t *it, double t0)
{
    seg_hdr_t ph;
    int fd;
    for (;;) {
        fd = shm_open(it->name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd >= 0 || errno != EEXIST) {
            break;
        }
        peek_hdr(it->name, &ph);
        if (ph.stamp == SHM_STAMP) {
            /* live, or in another pid namespace and not provably this job's
             * (an earlier incarnation of this very job is recycled) */
            const int state = owner_state(ph.owner, ph.pidns);
            if (state == 1 || (state < 0 && !(ph.job != 0 && ph.job == job_token()))) {
                fprintf(stderr, "ucg_builtin_shm_iface_open(%s): in use by %s process %llu "
                        "(another job with this name: set a job uid)\n", it->name,
                        state == 1 ? "live" : "another pid namespace's",
                        (unsigned long long)ph.owner);
                it->open_status = UCS_ERR_BUSY;
                return -1;
            }
        }
        /* a dead creator's object, a closed one, or one never set up */
        if (ph.stamp != 0 || now_s() - t0 > 1.0) {
            shm_unlink(it->name);
        } else {
            usleep(1000);
        }
    }
    if (fd < 0 || ftruncate(fd, (off_t)it->seg_bytes) != 0) {
        if (fd >= 0) {
            close(fd);
            shm_unlink(it->name);
        }
        it->open_status = UCS_ERR_IO_ERROR;
        return -1;
    }
    return fd;
}

static ucs_status_t iface_map(ucg_builtin_shm_iface_t *it)
{
    const double t0 = now_s(), lim = wait_timeout_s();
    struct stat stt;
    seg_hdr_t *h, ph;
    int fd;

    for (;;) {
        if (now_s() - t0 > lim) {
            fprintf(stderr, "ucg_builtin_shm_iface_open(%s): no usable object after %.0f s\n",
                    it->name, lim);
            it->open_status = UCS_ERR_TIMED_OUT;
            return it->open_status;
        }
        if (it->my == 0) {
            fd = iface_create(it, t0);
            if (fd < 0) {
                return it->open_status;
            }
        } else {
            fd = shm_open(it->name, O_RDWR, 0);
            if (fd >= 0 && (fstat(fd, &stt) != 0 || (size_t)stt.st_size < it->seg_bytes)) {
                close(fd);                          /* not sized yet */
                fd = -1;
            }
            if (fd < 0) {
                usleep(1000);                       /* member 0 has not made it yet */
                continue;
            }
        }
        it->seg = mmap(NULL, it->seg_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (it->seg == MAP_FAILED) {
            it->seg = NULL;
            it->open_status = UCS_ERR_NO_MEMORY;
            return it->open_status;
        }
        h = (seg_hdr_t*)it->seg;
        if (it->my == 0) {
            /* a fresh object is zero-filled: every ring starts empty */
            h->owner     = (uint64_t)getpid();
            h->instance  = random_u64();
            h->seg_bytes = it->seg_bytes;
            h->members   = it->members;
            h->pidns     = pid_ns();
            h->job       = job_token();
            member_attach(it);
            atomic_store_explicit(&h->stamp, SHM_STAMP, memory_order_release);
            return UCS_OK;
        }
        /* a peer: wait for the creator's stamp on this very object, unless
         * the name moves on to another one meanwhile */
        while (atomic_load_explicit(&h->stamp, memory_order_acquire) == 0 &&
               now_s() - t0 <= lim) {
            usleep(200);
            peek_hdr(it->name, &ph);
            if (ph.stamp == SHM_STAMP && ph.instance != h->instance) {
                break;
            }
        }
        if (atomic_load_explicit(&h->stamp, memory_order_acquire) == SHM_STAMP &&
            owner_state(h->owner, h->pidns) != 0 && foreign_job(h->job)) {
            fprintf(stderr, "ucg_builtin_shm_iface_open(%s): the object of another job "
                    "(creator %llu; set a job uid)\n", it->name,
                    (unsigned long long)h->owner);
            munmap(it->seg, it->seg_bytes);
            it->seg = NULL;
            it->open_status = UCS_ERR_BUSY;
            return it->open_status;
        }
        if (atomic_load_explicit(&h->stamp, memory_order_acquire) == SHM_STAMP &&
            owner_state(h->owner, h->pidns) != 0 && h->seg_bytes == it->seg_bytes &&
            h->members == it->members) {
            peek_hdr(it->name, &ph);
            if (ph.instance == h->instance) {
                member_attach(it);
                return UCS_OK;                      /* still the named object */
            }
        } else if (atomic_load_explicit(&h->stamp, memory_order_acquire) == SHM_STAMP &&
                   owner_state(h->owner, h->pidns) != 0) {
            fprintf(stderr, "ucg_builtin_shm_iface_open(%s): a live object of another "
                    "layout (%llu members, %llu B; here %u, %zu)\n", it->name,
                    (unsigned long long)h->members, (unsigned long long)h->seg_bytes,
                    it->members, it->seg_bytes);
            munmap(it->seg, it->seg_bytes);
            it->seg = NULL;
            it->open_status = UCS_ERR_BUSY;
            return it->open_status;
        }
        munmap(it->seg, it->seg_bytes);             /* stale or closed: again */
        it->seg = NULL;
        usleep(1000);
    }
}

ucs_status_t ucg_builtin_shm_iface_open(const char *name, unsigned members,
                                        unsigned my_index, size_t max_short,
                                        unsigned ring_cells,
                                        ucg_builtin_shm_iface_t **iface_p)
{
    ucg_builtin_shm_iface_t *it;
    ucs_status_t st;

    if (name == NULL || iface_p == NULL || members == 0 ||
        members > UCG_BUILTIN_OPS_MAX_MEMBERS || my_index >= members ||
        max_short <= 8 || max_short > (1u << 20) || ring_cells < 2) {
        return UCS_ERR_INVALID_PARAM;
    }
    it = calloc(1, sizeof(*it));
    if (it == NULL) {
        return UCS_ERR_NO_MEMORY;
    }
    {
        pthread_mutexattr_t a;
        pthread_mutexattr_init(&a);
        pthread_mutexattr_settype(&a, PTHREAD_MUTEX_RECURSIVE);
        pthread_mutex_init(&it->async_lock, &a);
        pthread_mutexattr_destroy(&a);
    }
    snprintf(it->name, sizeof(it->name), "/%s", name[0] == '/' ? name + 1 : name);
    it->members    = members;
    it->my         = my_index;
    it->max_short  = max_short;
    it->cells      = ring_cells;
    it->cell_size  = (sizeof(cell_t) + (max_short - 8) + 63) & ~(size_t)63;
    it->ring_bytes = sizeof(ring_ctl_t) + (size_t)ring_cells * it->cell_size;
    {
        /* UCX_BUILTIN_SM_INCAST=batched: a cell carries every child's message
         * side by side (the strided incast behind BATCHED_DATA receives,
         * builtin_comp_step.inl:242-273) */
        const char *e = getenv("UCX_BUILTIN_SM_INCAST");
        it->incast_batched = e && (e[0] == 'b' || e[0] == 'B');
    }
    it->incast_cell_size = (sizeof(incast_cell_t) +
                            (it->incast_batched ? members * max_short : max_short - 8) + 63) &
                           ~(size_t)63;
    it->incast_bytes     = sizeof(incast_ctl_t) + (size_t)ring_cells * it->incast_cell_size;
    it->ctl_bytes        = (SEG_HDR_BYTES + (size_t)members * sizeof(member_ctl_t) + 63) &
                           ~(size_t)63;
    it->incast_base      = it->ctl_bytes + (size_t)members * members * it->ring_bytes;
    it->seg_bytes        = it->incast_base + (size_t)members * it->incast_bytes;

    if (iface_map(it) != UCS_OK) {
        ucs_status_t st = it->open_status;
        pthread_mutex_destroy(&it->async_lock);
        free(it);
        return st;
    }
    st = ucg_builtin_shm_barrier(it);   /* everybody mapped before any send */
    if (st != UCS_OK) {
        (void)ucg_builtin_shm_iface_close(it);
        return st;
    }
    *iface_p = it;
    return UCS_OK;
}

/* A member whose peers are all there meets them at a last barrier, so that
 * none unmaps (member 0: unlinks) while another still sends. Once a peer is
 * gone, or a barrier already failed, the object is unmapped at once and the
 * failure returned: a drop-in component reports a peer's failure as a
 * status, it never kills its host process (the reference ends
 * ops with a status, builtin_comp_step.inl:332-333). The last member of a
 * dead creator's object unlinks it, if the name still refers to it. */
ucs_status_t ucg_builtin_shm_iface_close(ucg_builtin_shm_iface_t *it)
{
    seg_hdr_t *h, ph;
    ucs_status_t st;
    stash_t *m;
    if (it == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    h = (seg_hdr_t*)it->seg;
    if (it->my == 0) {
        /* closed before the last barrier: a member reopening the name at
         * once waits for the next instance (iface_map) */
        atomic_store_explicit(&h->stamp, SHM_CLOSED, memory_order_release);
    }
    st = ucg_builtin_shm_barrier(it);
    if (it->my == 0) {
        shm_unlink(it->name);
    } else if (st != UCS_OK && owner_state(h->owner, h->pidns) == 0) {
        peek_hdr(it->name, &ph);
        if (ph.instance == h->instance) {
            shm_unlink(it->name);
        }
    }
    munmap(it->seg, it->seg_bytes);
    while ((m = it->unexpected) != NULL) {
        it->unexpected = m->next;
        free(m);
    }
    pthread_mutex_destroy(&it->async_lock);
    free(it);
    return st;
}

size_t ucg_builtin_shm_iface_max_short(ucg_builtin_shm_iface_t *it)
{
    return it ? it->max_short : 0;
}

/* Every member arrives, or: a member's process is gone (probed while
 * waiting, UCS_ERR_CONNECTION_RESET), or the wait outlives
 * UCX_BUILTIN_WAIT_TIMEOUT (UCS_ERR_TIMED_OUT). After a failure the shared
 * count is out of step, so every later barrier of this member fails at once. */
ucs_status_t ucg_builtin_shm_barrier(ucg_builtin_shm_iface_t *it)
{
    _Atomic uint64_t *arrive;
    uint64_t gen;
    double t0, lim;
    unsigned spins = 0;
    if (it == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (broken_status(it) != UCS_OK) {
        return broken_status(it);
    }
    arrive = &((seg_hdr_t*)it->seg)->arrive;
    gen    = ++it->barrier_gen;
    t0     = now_s();
    lim    = wait_timeout_s();
    atomic_fetch_add_explicit(arrive, 1, memory_order_acq_rel);
    while (atomic_load_explicit(arrive, memory_order_acquire) < gen * it->members) {
        if ((++spins & 255) == 0) {
            if (shm_peer_check(it) >= 0) {
                return broken_status(it);
            }
            if (now_s() - t0 > lim) {
                fprintf(stderr, "ucg_builtin_shm_barrier(%s): timed out after %.0f s\n",
                        it->name, lim);
                return set_broken(it, UCS_ERR_TIMED_OUT);
            }
        }
        sched_yield();
    }
    return UCS_OK;
}

ucs_status_t ucg_builtin_shm_am_short(ucg_builtin_shm_iface_t *it, unsigned peer,
                                      uint64_t header, const void *payload,
                                      size_t length)
{
    ring_ctl_t *r;
    uint64_t head, tail;
    cell_t *c;

    if (peer >= it->members || peer == it->my) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (length + 8 > it->max_short) {
        return UCS_ERR_INVALID_PARAM;   /* UCS_ERR_MESSAGE_TRUNCATED in UCT */
    }
    r    = ring_ctl(it, it->my, peer);
    head = atomic_load_explicit(&r->head, memory_order_relaxed);
    tail = atomic_load_explicit(&r->tail, memory_order_acquire);
    if (head - tail >= it->cells) {
        return UCS_ERR_NO_RESOURCE;
    }
    c = ring_cell(it, r, head);
    c->length = (uint32_t)length;
    c->header = header;
    if (length) {
        memcpy(c + 1, payload, length);
    }
    atomic_store_explicit(&r->head, head + 1, memory_order_release);
    return UCS_OK;
}

/* the holder packs at most one fragment: spin briefly, then yield; a holder
 * that never lets go (its process is gone, or it outlives the wait timeout)
 * ends the send with a status */
static ucs_status_t spin_lock(ucg_builtin_shm_iface_t *it, _Atomic uint32_t *l)
{
    unsigned spins = 0;
    uint32_t z = 0;
    double t0 = 0.0;
    while (!atomic_compare_exchange_weak_explicit(l, &z, 1, memory_order_acquire,
                                                  memory_order_relaxed)) {
        z = 0;
        if (++spins < 256) {
            __builtin_ia32_pause();
            continue;
        }
        if (t0 == 0.0) {
            t0 = now_s();
        } else if ((spins & 1023) == 0) {
            if (shm_peer_check(it) >= 0) {
                return broken_status(it);
            }
            if (now_s() - t0 > wait_timeout_s()) {
                fprintf(stderr, "ucg_builtin_shm: incast cell lock held for over %.0f s\n",
                        wait_timeout_s());
                return UCS_ERR_TIMED_OUT;
            }
        }
        sched_yield();
    }
    return UCS_OK;
}

static void spin_unlock(_Atomic uint32_t *l)
{
    atomic_store_explicit(l, 0, memory_order_release);
}

ucs_status_t ucg_builtin_shm_am_incast(ucg_builtin_shm_iface_t *it, unsigned root,
                                       uint64_t header, unsigned expected,
                                       size_t length, ucg_builtin_pack_cb_f pack,
                                       void *arg, int concurrent)
{
    unsigned idx;
    incast_cell_t *c;
    ucs_status_t st;
    int first;

    if (root >= it->members || root == it->my || expected == 0 || pack == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (length + 8 > it->max_short) {
        return UCS_ERR_INVALID_PARAM;
    }
    /* the cell of this message: consecutive fragments of one message
     * (remote_offset in steps of at most max_short - 8) take consecutive
     * cells from a start that a multiplicative hash of the rest of the
     * header (group, coll_id, step) spreads out */
    idx = (unsigned)((((header & 0xffffffffull) * 0x9E3779B97F4A7C15ull) >> 40) +
                     (header >> 32) / (it->max_short - 8)) % it->cells;
    c   = incast_cell(it, root, idx);
    if ((st = spin_lock(it, &c->lock)) != UCS_OK) {
        return st;
    }
    /* acquire: the root's reads of a delivered cell precede our writes */
    if (atomic_load_explicit(&c->state, memory_order_acquire) == INCAST_FREE) {
        atomic_store_explicit(&c->state, INCAST_FILLING, memory_order_relaxed);
        atomic_store_explicit(&c->count, 0, memory_order_relaxed);
        c->header   = header;
        c->expected = expected;
        c->length   = (uint32_t)length;
        first       = 1;
    } else if (atomic_load_explicit(&c->state, memory_order_acquire) == INCAST_FILLING &&
               c->header == header) {
        first = 0;
    } else {
        spin_unlock(&c->lock);
        return UCS_ERR_NO_RESOURCE;   /* cell busy with another message */
    }
    if (concurrent) {
        /* atomic packers add into a zeroed cell outside the lock */
        if (first) {
            memset(c + 1, 0, length);
        }
        spin_unlock(&c->lock);
        pack(arg, c + 1, 1);
    } else {
        pack(arg, c + 1, !first);     /* first copies, the others reduce */
    }
    if (atomic_fetch_add_explicit(&c->count, 1, memory_order_acq_rel) + 1 == expected) {
        atomic_store_explicit(&c->state, INCAST_READY, memory_order_release);
        atomic_fetch_add_explicit(&incast_ctl(it, root)->ready, 1, memory_order_release);
    }
    if (!concurrent) {
        spin_unlock(&c->lock);
    }
    return UCS_OK;
}

/* The batched form: every child copies its message (header and payload)
 * into its own slot of the root's cell - slot k for the k-th to arrive - and
 * the root receives the cell as one message of `expected` (header, payload)
 * records, the first header being the cell's: [chunk 0][hdr 1][chunk 1]...
 * No child combines anything; the root reduces the chunks in slot order. */
ucs_status_t ucg_builtin_shm_am_incast_batched(ucg_builtin_shm_iface_t *it, unsigned root,
                                               uint64_t header, unsigned expected,
                                               const void *payload, size_t length)
{
    unsigned idx, k;
    incast_cell_t *c;
    ucs_status_t st;
    char *slot;

    if (root >= it->members || root == it->my || expected == 0 || !it->incast_batched ||
        expected >= it->members || length + 8 > it->max_short) {
        return UCS_ERR_INVALID_PARAM;
    }
    idx = (unsigned)((((header & 0xffffffffull) * 0x9E3779B97F4A7C15ull) >> 40) +
                     (header >> 32) / (it->max_short - 8)) % it->cells;
    c   = incast_cell(it, root, idx);
    if ((st = spin_lock(it, &c->lock)) != UCS_OK) {
        return st;
    }
    if (atomic_load_explicit(&c->state, memory_order_acquire) == INCAST_FREE) {
        atomic_store_explicit(&c->state, INCAST_FILLING, memory_order_relaxed);
        atomic_store_explicit(&c->count, 0, memory_order_relaxed);
        c->header   = header;
        c->expected = expected;
        c->length   = (uint32_t)length;
        c->reserved = 0;                     /* slots handed out */
    } else if (!(atomic_load_explicit(&c->state, memory_order_acquire) == INCAST_FILLING &&
                 c->header == header)) {
        spin_unlock(&c->lock);
        return UCS_ERR_NO_RESOURCE;          /* cell busy with another message */
    }
    k = c->reserved++;
    spin_unlock(&c->lock);
    slot = (char*)(c + 1) + (size_t)k * (length + 8);
    if (k) {
        memcpy(slot - 8, &header, 8);
    }
    memcpy(slot, payload, length);
    if (atomic_fetch_add_explicit(&c->count, 1, memory_order_acq_rel) + 1 == expected) {
        atomic_store_explicit(&c->state, INCAST_READY, memory_order_release);
        atomic_fetch_add_explicit(&incast_ctl(it, root)->ready, 1, memory_order_release);
    }
    return UCS_OK;
}

static unsigned incast_progress(ucg_builtin_shm_iface_t *it, ucg_builtin_am_cb_f cb,
                                void *arg)
{
    incast_ctl_t *ctl = incast_ctl(it, it->my);
    unsigned i, n = 0;
    if (atomic_load_explicit(&ctl->ready, memory_order_acquire) == 0) {
        return 0;
    }
    for (i = 0; i < it->cells; i++) {
        incast_cell_t *c = incast_cell(it, it->my, i);
        if (atomic_load_explicit(&c->state, memory_order_acquire) != INCAST_READY) {
            continue;
        }
        (void)cb(arg, &c->header, it->incast_batched ?
                                  (size_t)c->expected * (8 + (size_t)c->length) :
                                  8 + (size_t)c->length);
        atomic_fetch_sub_explicit(&ctl->ready, 1, memory_order_relaxed);
        atomic_store_explicit(&c->state, INCAST_FREE, memory_order_release);
        n++;
    }
    return n;
}

unsigned ucg_builtin_shm_progress(ucg_builtin_shm_iface_t *it,
                                  ucg_builtin_am_cb_f cb, void *arg)
{
    unsigned src, n = incast_progress(it, cb, arg);
    for (src = 0; src < it->members; src++) {
        ring_ctl_t *r;
        uint64_t tail, head;
        if (src == it->my) {
            continue;
        }
        r    = ring_ctl(it, src, it->my);
        tail = atomic_load_explicit(&r->tail, memory_order_relaxed);
        head = atomic_load_explicit(&r->head, memory_order_acquire);
        while (tail < head) {
            cell_t *c = ring_cell(it, r, tail);
            (void)cb(arg, &c->header, 8 + (size_t)c->length);
            tail++;
            /* the cell is free only after the callback returned */
            atomic_store_explicit(&r->tail, tail, memory_order_release);
            n++;
        }
    }
    return n;
}
