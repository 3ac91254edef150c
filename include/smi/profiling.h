/*
 * profiling.h -- live per-kernel timing with HIP events.
 *
 * The reference times whole kernel sets with std::chrono or OpenCL events
 * (examples/host/stencil_smi.cpp:316-340, microbenchmarks/host/
 * reduce_benchmark.cpp:120-155).  Here, while enabled, every launch of the
 * named hot kernel is bracketed by a pair of hipEvents recorded on the
 * stream it is launched on; smi_prof_read returns the summed duration.
 */
#ifndef SMI_PROFILING_H
#define SMI_PROFILING_H

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    SMI_PROF_STENCIL_SWEEP = 0,  /* the Jacobi sweep kernel                */
    SMI_PROF_STENCIL_EDGE = 1,   /* halo-edge kernel (multi-rank overlap)  */
    SMI_PROF_REDUCE_FOLD = 2,
    SMI_PROF_GEMV = 3,
    SMI_PROF_STENCIL_SWEEPK = 4, /* the K-step (temporally blocked) sweep  */
    SMI_PROF_KMEANS_ASSIGN = 5,  /* kmeans ComputeDistance                 */
    SMI_PROF_KMEANS_FOLD = 6,    /* kmeans per-cluster sum chains          */
    SMI_PROF_NUM = 7
} SMI_ProfKernel;

int smi_prof_enable(int enable);
int smi_prof_reset(void);
/* Synchronises the recorded events; *total_ms = summed kernel time,
 * *launches = number of timed launches of `kernel`. */
int smi_prof_read(int kernel, double *total_ms, long *launches);
/* The same for launches recorded with `tag` (-1: any tag; the K-step sweep
 * tags each launch with its K); *units (nullable) = their summed
 * algorithmic work: cell-steps for the stencil kernels. */
int smi_prof_read_tag(int kernel, int tag, double *total_ms, long *launches, double *units);
/* Distinct (kernel, tag) pairs recorded since the last reset, in first-seen
 * order: up to max_entries written, *n_entries = how many exist. */
int smi_prof_list(int *kernels, int *tags, int max_entries, int *n_entries);

#ifdef __cplusplus
}
#endif
#endif /* SMI_PROFILING_H */
