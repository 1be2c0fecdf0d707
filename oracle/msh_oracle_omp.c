/*
 * msh_oracle_omp.c — ORACLE, TEST INFRASTRUCTURE ONLY (see msh_oracle.c header).
 *
 * Pod-parallel driver of the same scalar restatement, used only as the multi-core CPU
 * baseline in bench.py ("C++ oracle: 1 thread, and OpenMP on all host
 * cores"). Pods are independent in the batched mode (no plugin reads placement state),
 * so a static split over threads gives the identical results.
 */
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#include "msh_oracle.h"

int oracle_schedule_batch_soa_omp(int32_t n, const uint8_t* unsched, const int8_t* node_digit,
                                  int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                                  const int32_t* filter_ids, int32_t nf,
                                  const int32_t* prescore_ids, int32_t npre,
                                  const int32_t* score_ids, const int64_t* weights,
                                  const int32_t* norm, int32_t ns, int32_t threads,
                                  int32_t* out_idx, int64_t* out_score, int32_t* out_status) {
  if (p < 0 || threads < 1) return -1;
  int rc_all = 0;
#pragma omp parallel num_threads(threads) reduction(| : rc_all)
  {
    int t = omp_get_thread_num(), nt = omp_get_num_threads();
    int32_t lo = (int32_t)((int64_t)p * t / nt), hi = (int32_t)((int64_t)p * (t + 1) / nt);
    if (hi > lo) {
      rc_all |= oracle_schedule_soa_impl(n, unsched, node_digit, hi - lo, pod_digit + lo,
                                         pod_tol + lo, filter_ids, nf, prescore_ids, npre,
                                         score_ids, weights, norm, ns, 0, 0, 0, NULL, NULL,
                                         out_idx + lo, out_score + lo, out_status + lo, NULL);
    }
  }
  return rc_all ? -1 : 0;
}

/* The same pod-parallel split for plugin lists with score-column plugins (cols: the columns, List
 * order, column k at cols + k * n). */
int oracle_schedule_batch_soa_cols_omp(int32_t n, const uint8_t* unsched, const int8_t* node_digit,
                                       int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                                       const int32_t* filter_ids, int32_t nf,
                                       const int32_t* prescore_ids, int32_t npre,
                                       const int32_t* score_ids, const int64_t* weights,
                                       const int32_t* norm, int32_t ns, const int64_t* cols,
                                       int32_t threads, int32_t* out_idx, int64_t* out_score,
                                       int32_t* out_status) {
  if (p < 0 || threads < 1) return -1;
  int rc_all = 0;
#pragma omp parallel num_threads(threads) reduction(| : rc_all)
  {
    int t = omp_get_thread_num(), nt = omp_get_num_threads();
    int32_t lo = (int32_t)((int64_t)p * t / nt), hi = (int32_t)((int64_t)p * (t + 1) / nt);
    if (hi > lo) {
      rc_all |= oracle_schedule_soa_impl(n, unsched, node_digit, hi - lo, pod_digit + lo,
                                         pod_tol + lo, filter_ids, nf, prescore_ids, npre,
                                         score_ids, weights, norm, ns, 0, 0, 0, NULL, cols,
                                         out_idx + lo, out_score + lo, out_status + lo, NULL);
    }
  }
  return rc_all ? -1 : 0;
}
