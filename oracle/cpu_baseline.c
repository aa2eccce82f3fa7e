/*
 * cpu_baseline.c -- times the oracle's fp32 MPI_SUM loop on host cores.
 * TEST / BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * The loop is the reference's MPIR_OP_TYPE_REDUCE_CASE body for MPI_FLOAT
 * with MPIR_LSUM (mpir_op_util.h:48-55, opsum.c:15), compiled like MPICH
 * (gcc -O2, configure.ac:399-408), run by oracle_reduce_local_nocheck.
 * Each thread owns its own (inbuf, inoutbuf) pair of `count` floats and
 * performs `iters` calls; the figure reported is the aggregate algorithmic
 * rate 3 * count * 4 * iters * nthreads / (slowest thread's wall time).
 *
 * oracle_cpu_baseline_sum_f32_pinned: the same, one thread pinned to each
 * listed CPU (bench.py passes one logical CPU per physical core), pages
 * first-touched by the pinned owner (so NUMA-local under Linux's first-touch
 * policy), all threads released together by a barrier before the timed
 * calls; per-thread seconds are returned for per-socket figures.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

int oracle_reduce_local_nocheck(const void *inbuf, void *inoutbuf, int count, int datatype, int op);

typedef struct {
    long count;
    int iters;
    double seconds;
    int rc;
    int cpu;                    /* -1: not pinned */
    pthread_barrier_t *bar;     /* NULL: start as soon as ready */
} job_t;

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void *worker(void *arg)
{
    job_t *j = (job_t *) arg;
    float *in = malloc((size_t) j->count * 4), *io = malloc((size_t) j->count * 4);
    long i;
    int it;
    double t0;
    if (!in || !io) {
        j->rc = -1;
        free(in);
        free(io);
        if (j->bar)
            pthread_barrier_wait(j->bar);
        return NULL;
    }
    if (j->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(j->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    for (i = 0; i < j->count; i++) {    /* first touch by the owning thread */
        in[i] = (float) (i % 1000) * 1e-3f;
        io[i] = (float) (i % 977) * 0.5f;
    }
    /* one untimed warm-up call */
    oracle_reduce_local_nocheck(in, io, (int) j->count, 0x4c00040a, 0x58000003);
    if (j->bar)
        pthread_barrier_wait(j->bar);
    t0 = now();
    for (it = 0; it < j->iters; it++)
        oracle_reduce_local_nocheck(in, io, (int) j->count, 0x4c00040a, 0x58000003);
    j->seconds = now() - t0;
    j->rc = 0;
    free(in);
    free(io);
    return NULL;
}

/* returns the slowest thread's seconds, or < 0 on failure */
double oracle_cpu_baseline_sum_f32(int nthreads, long count, int iters)
{
    pthread_t *th = calloc(nthreads, sizeof(pthread_t));
    job_t *jobs = calloc(nthreads, sizeof(job_t));
    double worst = 0;
    int t;
    for (t = 0; t < nthreads; t++) {
        jobs[t].count = count;
        jobs[t].iters = iters;
        jobs[t].cpu = -1;
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc)
            worst = -1;
        else if (worst >= 0 && jobs[t].seconds > worst)
            worst = jobs[t].seconds;
    }
    free(th);
    free(jobs);
    return worst;
}

/* pinned, barrier-started; seconds[t] per thread; returns the slowest, < 0 on failure */
double oracle_cpu_baseline_sum_f32_pinned(int nthreads, const int *cpus, long count, int iters, double *seconds)
{
    pthread_t *th = calloc(nthreads, sizeof(pthread_t));
    job_t *jobs = calloc(nthreads, sizeof(job_t));
    pthread_barrier_t bar;
    double worst = 0;
    int t;
    pthread_barrier_init(&bar, NULL, (unsigned) nthreads);
    for (t = 0; t < nthreads; t++) {
        jobs[t].count = count;
        jobs[t].iters = iters;
        jobs[t].cpu = cpus[t];
        jobs[t].bar = &bar;
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        seconds[t] = jobs[t].rc ? -1.0 : jobs[t].seconds;
        if (jobs[t].rc)
            worst = -1;
        else if (worst >= 0 && jobs[t].seconds > worst)
            worst = jobs[t].seconds;
    }
    pthread_barrier_destroy(&bar);
    free(th);
    free(jobs);
    return worst;
}
