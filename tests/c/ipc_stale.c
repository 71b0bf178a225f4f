/*
 * ipc_stale.c - is a peer's device buffer, read through an IPC mapping by
 * another process on the same GPU, current once the writer's kernel has
 * completed and the writer has said so? The engine's remote-key steps
 * (builtin_ops.c) rely on it: a member reads its senders' buffers after their
 * READY, and the same registered buffers carry new data in every op.
 *
 *   RANK=0|1 WORLD_SIZE=2 ipc_stale <shm-name> [iters=500] [bytes=65536] [read=kernel|dma]
 *
 * Rank 0 owns buffer X: for each i it writes pattern i into X with a kernel
 * (the synthetic generator, seed i), waits for the stream and sends READY i.
 * Rank 1 maps X once, and for each READY copies X into a local buffer - with
 * a kernel through its L2s (read=kernel) or with the copy engine (read=dma) -
 * downloads it, compares it with pattern i generated on the host (the oracle,
 * test infrastructure) and answers DONE i. Rank 1 prints one JSON line with
 * the number of iterations that saw data other than pattern i.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ucg_builtin_ops.h"
#include "combine_ref.h"

static uint64_t g_hdr;
static uint8_t g_payload[256];
static int g_got;

static ucs_status_t on_msg(void *arg, void *data, size_t length)
{
    (void)arg;
    memcpy(&g_hdr, data, 8);
    memcpy(g_payload, (char*)data + 8, length - 8);
    g_got = 1;
    return UCS_OK;
}

static uint64_t wait_msg(ucg_builtin_shm_iface_t *it)
{
    g_got = 0;
    while (!g_got) {
        ucg_builtin_shm_progress(it, on_msg, NULL);
    }
    return g_hdr;
}

static void send_msg(ucg_builtin_shm_iface_t *it, unsigned peer, uint64_t hdr,
                     const void *p, size_t n)
{
    while (ucg_builtin_shm_am_short(it, peer, hdr, p, n) == UCS_ERR_NO_RESOURCE) {
    }
}

int main(int argc, char **argv)
{
    const char *name = argc > 1 ? argv[1] : "/ucg_ipc_stale";
    int iters        = argc > 2 ? atoi(argv[2]) : 500;
    size_t bytes     = argc > 3 ? (size_t)atol(argv[3]) : 65536;
    int dma          = argc > 4 && strcmp(argv[4], "dma") == 0;
    unsigned rank    = (unsigned)atoi(getenv("RANK") ? getenv("RANK") : "0");
    size_t n = bytes / 4;
    ucg_builtin_dev_ctx_params_t prm = {0, NULL, 0, 0, 0, 0};
    ucg_builtin_dev_ctx_t *ctx;
    ucg_builtin_shm_iface_t *it;
    uint8_t key[UCG_BUILTIN_DEV_IPC_HANDLE_BYTES];
    int i, stale = 0, first = -1;

    if (ucg_builtin_dev_ctx_create(&prm, &ctx) != UCS_OK ||
        ucg_builtin_shm_iface_open(name, 2, rank, 256, 16, &it) != UCS_OK) {
        fprintf(stderr, "set-up failed: %s\n", ucg_builtin_dev_last_error());
        return 1;
    }
    if (rank == 0) {
        const char *we = getenv("IPC_STALE_WAIT");
        const int wait_signal = we && strcmp(we, "signal") == 0;
        void *x = ucg_builtin_dev_malloc(ctx, bytes);
        if (x == NULL || ucg_builtin_dev_ipc_export(ctx, x, key) != UCS_OK) {
            return 1;
        }
        send_msg(it, 1, 1, key, sizeof(key));
        for (i = 0; i < iters; i++) {
            ucg_builtin_dev_fill(ctx, UCG_DEV_DT_UINT32, UCG_DEV_DIST_ROUND,
                                 0x5A1E0000u + i, x, n);
            /* IPC_STALE_WAIT=signal: the engine's wait (the pinned completion
             * word), else the runtime's hipStreamSynchronize */
            if (wait_signal) {
                ucg_builtin_dev_complete(ctx);
            } else {
                ucg_builtin_dev_sync(ctx);
            }
            send_msg(it, 1, 2 + (uint64_t)i, NULL, 0);
            if (wait_msg(it) != 2 + (uint64_t)i) {
                fprintf(stderr, "rank 0: out of step at %d\n", i);
                return 1;
            }
        }
        ucg_builtin_shm_barrier(it);
        ucg_builtin_dev_free(ctx, x);
    } else {
        void *xp = NULL, *local = ucg_builtin_dev_malloc(ctx, bytes);
        uint32_t *got = malloc(bytes), *want = malloc(bytes);
        if (wait_msg(it) != 1 ||
            ucg_builtin_dev_ipc_import(ctx, g_payload, &xp) != UCS_OK) {
            fprintf(stderr, "rank 1: import failed: %s\n", ucg_builtin_dev_last_error());
            return 1;
        }
        for (i = 0; i < iters; i++) {
            void *const d[1] = {local};
            const void *const s[1] = {xp};
            if (wait_msg(it) != 2 + (uint64_t)i) {
                fprintf(stderr, "rank 1: out of step at %d\n", i);
                return 1;
            }
            if (dma) {
                ucg_builtin_dev_memcpy(ctx, local, xp, bytes);
            } else {
                ucg_builtin_dev_copy_multi(ctx, d, s, 1, bytes);
                ucg_builtin_dev_sync(ctx);
            }
            ucg_builtin_dev_memcpy(ctx, got, local, bytes);
            ucg_oracle_fill(ORA_U32, ORA_DIST_ROUND, 0x5A1E0000u + i, want, n);
            if (memcmp(got, want, bytes)) {
                stale++;
                if (first < 0) {
                    first = i;
                }
            }
            send_msg(it, 0, 2 + (uint64_t)i, NULL, 0);
        }
        printf("{\"probe\": \"ipc_stale\", \"read\": \"%s\", \"bytes\": %zu, \"iters\": %d, "
               "\"stale_iters\": %d, \"first_stale\": %d}\n", dma ? "dma" : "kernel", bytes,
               iters, stale, first);
        ucg_builtin_shm_barrier(it);
        ucg_builtin_dev_ipc_release(ctx, xp);
        ucg_builtin_dev_free(ctx, local);
        free(got);
        free(want);
    }
    ucg_builtin_shm_iface_close(it);
    ucg_builtin_dev_ctx_destroy(ctx);
    return stale ? 3 : 0;
}
