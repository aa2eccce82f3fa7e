// clock_cost.c -- cost of the clocks a hot path might read on this host:
// clock_gettime(CLOCK_MONOTONIC / _RAW / _COARSE) and rdtsc, ns per call.
//   gcc -O2 -o tools/clock_cost tools/clock_cost.c
#include <stdio.h>
#include <stdint.h>
#include <time.h>
#include <x86intrin.h>
static double now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec * 1e9 + t.tv_nsec; }
int main(void) {
    const int n = 200000;
    const clockid_t ids[] = {CLOCK_MONOTONIC, CLOCK_MONOTONIC_RAW, CLOCK_MONOTONIC_COARSE, CLOCK_REALTIME};
    const char *names[] = {"CLOCK_MONOTONIC", "CLOCK_MONOTONIC_RAW", "CLOCK_MONOTONIC_COARSE", "CLOCK_REALTIME"};
    for (int k = 0; k < 4; ++k) {
        struct timespec t;
        double t0 = now();
        for (int i = 0; i < n; ++i) clock_gettime(ids[k], &t);
        printf("%-24s %8.1f ns per call\n", names[k], (now() - t0) / n);
    }
    double t0 = now();
    uint64_t s = 0;
    for (int i = 0; i < n; ++i) s += __rdtsc();
    printf("%-24s %8.1f ns per call (%llu)\n", "rdtsc", (now() - t0) / n, (unsigned long long)(s & 1));
    FILE *f = fopen("/sys/devices/system/clocksource/clocksource0/current_clocksource", "r");
    char buf[64] = "?";
    if (f) { if (!fgets(buf, sizeof buf, f)) buf[0] = 0; fclose(f); }
    printf("clocksource: %s", buf);
    return 0;
}
