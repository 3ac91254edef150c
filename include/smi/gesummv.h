/*
 * gesummv.h -- the gesummv_smi hot path: y = alpha*A*x + beta*B*x.
 *
 * Replaces the row-streamed `gemv` kernels of
 * examples/kernels/gesummv_rank0.cl:53-181 / gesummv_rank1.cl:50-187, the
 * rank-1 SMI_Push of beta*B*x and rank-0 `axpy` (gesummv_rank0.cl:184-203).
 * Fold contract per row (gesummv_rank0.cl:111-171):
 *   c_k = sequential fp32 sum of 64 products a*x (mul then add, no FMA)
 *   per 128-column tile: acc = (0 + alpha*c_{2t}) + alpha*c_{2t+1}
 *   y_row = ((0 + acc_0) + acc_1) + ...      (same with beta for B)
 *   y = yA + yB
 * m must be a multiple of 64 (gesummv_rank0.cl:268).
 */
#ifndef SMI_GESUMMV_H
#define SMI_GESUMMV_H

#include "communicator.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Local kernel: y[i] = fold(A_i, alpha) + fold(B_i, beta) for the n rows of
 * this rank (A and B row-major with leading dimension lda >= m).  Pass
 * B = NULL for the single-matrix GEMV y[i] = fold(A_i, alpha). */
int smi_gemv_rows(const float *A, const float *B, const float *x, float *y,
                  int n, int m, int lda, float alpha, float beta,
                  SMI_Stream stream);

/* Distributed gesummv: the n_global rows are sharded contiguously over the
 * ranks of `comm` (rank r owns rows [r*n_global/size, (r+1)*n_global/size));
 * every rank holds its rows of A and B and the whole x; the partial y chunks
 * are streamed to `root`, whose y (n_global elements) receives the result. */
int smi_gesummv(SMI_Comm comm, const float *A_rows, const float *B_rows,
                const float *x, float *y, int n_global, int m, float alpha,
                float beta, int root, SMI_Stream stream);

#ifdef __cplusplus
}
#endif
#endif /* SMI_GESUMMV_H */
