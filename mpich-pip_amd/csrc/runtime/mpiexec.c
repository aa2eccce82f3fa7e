/*
 * mpiexec.c -- single-node launcher for the runtime subset (config 1:
 * `mpiexec -n 2 examples/cpi`).  Stands in for Hydra + PMI + pip_spawn
 * (src/pm/hydra, pmip_cb.c:485-497): creates the shared world segment
 * (pip_shm.h), forks N ranks that exec the program with MPIR_PIP_RANK /
 * MPIR_PIP_SIZE / MPIR_PIP_SHM set, waits for them, and tears the world
 * down.  When a rank fails (non-zero exit or a signal) the others are
 * terminated, as Hydra does; the exit status is the first failure's.
 *
 *   mpiexec -n N [--timeout SECONDS] program [args...]
 *   (MPIEXEC_TIMEOUT in the environment is honoured like Hydra's.)
 *
 * The launcher never touches a GPU: ranks initialise HIP themselves after
 * exec.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "pip_shm.h"

static pid_t pids[PIP_MAX_RANKS];
static int nranks;
static volatile sig_atomic_t timed_out;

static void on_alarm(int sig)
{
    (void) sig;
    timed_out = 1;
}

static void kill_all(int sig)
{
    int i;
    for (i = 0; i < nranks; i++)
        if (pids[i] > 0)
            kill(pids[i], sig);
}

static void usage(void)
{
    fprintf(stderr, "usage: mpiexec -n N [--timeout SECONDS] program [args...]\n");
    exit(2);
}

int main(int argc, char **argv)
{
    int i, a = 1, timeout = 0, status = 0, live, fd;
    char name[64], buf[16];
    size_t bytes;
    pip_shm_t *shm;
    const char *et = getenv("MPIEXEC_TIMEOUT");
    if (et)
        timeout = atoi(et);
    nranks = 1;
    while (a < argc && argv[a][0] == '-') {
        if ((!strcmp(argv[a], "-n") || !strcmp(argv[a], "-np")) && a + 1 < argc) {
            nranks = atoi(argv[a + 1]);
            a += 2;
        } else if (!strcmp(argv[a], "--timeout") && a + 1 < argc) {
            timeout = atoi(argv[a + 1]);
            a += 2;
        } else if (!strcmp(argv[a], "--")) {
            a++;
            break;
        } else {
            usage();
        }
    }
    if (a >= argc || nranks < 1 || nranks > PIP_MAX_RANKS)
        usage();

    snprintf(name, sizeof(name), "/mpich_pip_amd.%d.%ld", (int) getpid(), (long) time(NULL));
    bytes = PIP_SEGMENT_BYTES(nranks);
    fd = shm_open(name, O_RDWR | O_CREAT | O_EXCL, 0600);
    if (fd < 0 || ftruncate(fd, (off_t) bytes) != 0) {
        fprintf(stderr, "mpiexec: cannot create shared segment %s: %s\n", name, strerror(errno));
        return 1;
    }
    shm = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (shm == MAP_FAILED) {
        shm_unlink(name);
        fprintf(stderr, "mpiexec: mmap: %s\n", strerror(errno));
        return 1;
    }
    memset(shm, 0, PIP_DATA_OFFSET);
    shm->size = (uint32_t) nranks;
    shm->magic = PIP_MAGIC;
    munmap(shm, bytes);

    fflush(NULL);
    for (i = 0; i < nranks; i++) {
        pid_t p = fork();
        if (p < 0) {
            fprintf(stderr, "mpiexec: fork: %s\n", strerror(errno));
            kill_all(SIGKILL);
            status = 1;
            nranks = i;
            break;
        }
        if (p == 0) {
            snprintf(buf, sizeof(buf), "%d", i);
            setenv("MPIR_PIP_RANK", buf, 1);
            snprintf(buf, sizeof(buf), "%d", nranks);
            setenv("MPIR_PIP_SIZE", buf, 1);
            setenv("MPIR_PIP_SHM", name, 1);
            /* AQL rings in device memory unless the user chose otherwise: the CP
             * reads each dispatch packet from VRAM, not over PCIe, 1.4 us off every
             * synchronous MPI_Reduce_local (Synchronous return); ranks
             * exec before the HSA runtime starts, so it applies */
            setenv("HSA_ALLOCATE_QUEUE_DEV_MEM", "1", 0);
            execvp(argv[a], argv + a);
            fprintf(stderr, "mpiexec: cannot execute %s: %s\n", argv[a], strerror(errno));
            _exit(127);
        }
        pids[i] = p;
    }

    if (timeout > 0) {
        struct sigaction sa;
        memset(&sa, 0, sizeof(sa));
        sa.sa_handler = on_alarm;       /* no SA_RESTART: waitpid must return EINTR */
        sigaction(SIGALRM, &sa, NULL);
        alarm((unsigned) timeout);
    }
    live = nranks;
    while (live > 0) {
        int st;
        pid_t p = waitpid(-1, &st, 0);
        if (p < 0) {
            if (errno == EINTR && timed_out) {
                fprintf(stderr, "mpiexec: timeout after %d s, terminating ranks\n", timeout);
                kill_all(SIGKILL);
                if (!status)
                    status = 124;
                timed_out = 0;
                continue;
            }
            if (errno == EINTR)
                continue;
            break;
        }
        for (i = 0; i < nranks; i++)
            if (pids[i] == p) {
                pids[i] = 0;
                live--;
            }
        if (WIFEXITED(st) && WEXITSTATUS(st) != 0) {
            if (!status)
                status = WEXITSTATUS(st);
            kill_all(SIGTERM);
        } else if (WIFSIGNALED(st)) {
            if (!status)
                status = 128 + WTERMSIG(st);
            kill_all(SIGTERM);
        }
    }
    shm_unlink(name);
    return status;
}
