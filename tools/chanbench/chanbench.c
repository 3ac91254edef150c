/* chanbench.c -- throughput of the element-granular channel API, the way a C
 * host of the reference drives it (one SMI_Push / SMI_Pop call per element,
 * examples/host + microbenchmarks/kernels/bandwidth_0.cl:13-35 shape), over
 * the in-process transport on one GPU: rank 0 pushes N elements to rank 1
 * (two host threads).  Also SMI_Reduce element streams (4 ranks, int add;
 * 8 ranks, fp32 add with the reference's n * i known answer) and a SMI_Bcast
 * stream.  Prints one JSON line per measurement.
 *
 *   chanbench [N] */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "smi.h"

static int g_group, g_n;
static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef struct {
    int rank, world, mode, ad;
    double secs;
    long bad;
} Arg;

static void *rank_main(void *p) {
    Arg *a = (Arg *)p;
    SMI_Comm comm;
    if (smi_init_local(g_group, a->rank, 0, &comm) != 0) {
        fprintf(stderr, "init: %s\n", smi_last_error());
        exit(2);
    }
    const double t0 = now();
    if (a->mode == 0) { /* p2p 0 -> 1 */
        if (a->rank == 0) {
            SMI_Channel c = a->ad ? SMI_Open_send_channel_ad(g_n, SMI_INT, 1, 0, comm, a->ad)
                                  : SMI_Open_send_channel(g_n, SMI_INT, 1, 0, comm);
            for (int i = 0; i < g_n; ++i) SMI_Push(&c, &i);
        } else if (a->rank == 1) {
            SMI_Channel c = a->ad ? SMI_Open_receive_channel_ad(g_n, SMI_INT, 0, 0, comm, a->ad)
                                  : SMI_Open_receive_channel(g_n, SMI_INT, 0, 0, comm);
            for (int i = 0; i < g_n; ++i) {
                int v;
                SMI_Pop(&c, &v);
                a->bad += v != i;
            }
        }
    } else if (a->mode == 1) { /* bcast from rank 0 */
        SMI_BChannel c = SMI_Open_bcast_channel(g_n, SMI_FLOAT, 1, 0, comm);
        for (int i = 0; i < g_n; ++i) {
            float v = (float)i;
            SMI_Bcast(&c, &v);
            a->bad += v != (float)i;
        }
    } else if (a->mode == 2) { /* element reduce to rank 0 */
        SMI_RChannel c = SMI_Open_reduce_channel(g_n, SMI_INT, SMI_ADD, 2, 0, comm);
        for (int i = 0; i < g_n; ++i) {
            int s = i + a->rank, r = 0;
            SMI_Reduce(&c, &s, &r);
            if (a->rank == 0) a->bad += r != a->world * i + a->world * (a->world - 1) / 2;
        }
    } else { /* fp32 element reduce to the last rank: test/reduce/reduce.cl:17-20 KAT, n * i exact */
        const int root = a->world - 1;
        SMI_RChannel c = SMI_Open_reduce_channel(g_n, SMI_FLOAT, SMI_ADD, 3, root, comm);
        for (int i = 0; i < g_n; ++i) {
            float s = (float)(i & 0xffff), r = 0.f;
            SMI_Reduce(&c, &s, &r);
            if (a->rank == root) a->bad += r != (float)a->world * (float)(i & 0xffff);
        }
    }
    a->secs = now() - t0;
    smi_finalize(comm);
    return NULL;
}

static void run(const char *what, int world, int mode, int ad) {
    if (smi_local_group_create(world, &g_group) != 0) {
        fprintf(stderr, "group: %s\n", smi_last_error());
        exit(2);
    }
    pthread_t th[8];
    Arg a[8];
    for (int r = 0; r < world; ++r) {
        a[r] = (Arg){r, world, mode, ad, 0.0, 0};
        pthread_create(&th[r], NULL, rank_main, &a[r]);
    }
    double secs = 0;
    long bad = 0;
    for (int r = 0; r < world; ++r) {
        pthread_join(th[r], NULL);
        if (a[r].secs > secs) secs = a[r].secs;
        bad += a[r].bad;
    }
    printf("{\"channel\": \"%s\", \"ranks\": %d, \"asynch_degree\": %d, \"elements\": %d, \"s\": %.4f, "
           "\"Melem_per_s\": %.3f, \"MB_per_s\": %.2f, \"mismatches\": %ld}\n",
           what, world, ad, g_n, secs, g_n / secs / 1e6, g_n * 4.0 / secs / 1e6, bad);
    fflush(stdout);
    if (bad) exit(1);
}

int main(int argc, char **argv) {
    g_n = argc > 1 ? atoi(argv[1]) : 1000000;
    run("SMI_Push/SMI_Pop int", 2, 0, 0);
    run("SMI_Push/SMI_Pop int", 2, 0, 64);
    run("SMI_Push/SMI_Pop int", 2, 0, 1);
    run("SMI_Bcast float", 4, 1, 0);
    run("SMI_Reduce int add", 4, 2, 0);
    run("SMI_Reduce float add", 8, 3, 0);
    return 0;
}
