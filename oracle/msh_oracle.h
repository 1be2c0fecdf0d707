/* msh_oracle.h — ORACLE (test infrastructure only; see msh_oracle.c header). */
#ifndef MSH_ORACLE_H
#define MSH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_MAX_PLUGINS 8

enum { ORACLE_PLACED = 0, ORACLE_FIT_ERROR = 1, ORACLE_SCORE_ERROR = 2 };
enum { ORACLE_PLUGIN_NODE_UNSCHEDULABLE = 1, ORACLE_PLUGIN_NODE_NUMBER = 2 };
/* Score-column plugins (build extension, MSH_PLUGIN_SCORE_COLUMN0..3 of the C-ABI): Score(pod, node)
 * = a host-computed int64 per node, column k of oracle_nodes.cols. */
#define ORACLE_PLUGIN_SCORE_COLUMN0 16
#define ORACLE_MAX_COLUMNS 4
enum {
  ORACLE_NORM_NONE = 0,
  ORACLE_NORM_DEFAULT = 1,
  ORACLE_NORM_DEFAULT_REVERSE = 2,
  ORACLE_NORM_MINMAX = 3
};

typedef struct {
  int32_t n;
  const uint8_t* unsched; /* node.Spec.Unschedulable, List order */
  const int8_t* digit;    /* Atoi(last byte of node.Name) or -1 */
  const int64_t* cols;    /* ORACLE_MAX_COLUMNS x n score columns (column k at cols + k*n), or NULL */
} oracle_nodes;

typedef struct {
  int8_t digit;      /* Atoi(last byte of pod.Name) or -1 */
  uint8_t tolerates; /* tolerations tolerate the unschedulable taint */
} oracle_pod;

typedef struct {
  int32_t nf, npre, ns;
  int32_t filter_ids[ORACLE_MAX_PLUGINS];
  int32_t prescore_ids[ORACLE_MAX_PLUGINS];
  int32_t score_ids[ORACLE_MAX_PLUGINS];
  int64_t weights[ORACLE_MAX_PLUGINS];
  int32_t normalize[ORACLE_MAX_PLUGINS];
} oracle_plugins;

typedef struct {
  int32_t idx;    /* selected node index or -1 */
  int64_t score;  /* total score of the selected node */
  int32_t status; /* ORACLE_PLACED / FIT_ERROR / SCORE_ERROR */
  uint32_t diag;  /* FitError: Diagnosis.UnschedulablePlugins as a bitmask over filter slots */
} oracle_result;

int oracle_workspace_bytes(int32_t n_nodes, int32_t ns, size_t* out);
int oracle_schedule_batch(const oracle_nodes* nodes, const oracle_pod* pods, int32_t p,
                          const oracle_plugins* pl, int norm_in_loop, oracle_result* out);
int oracle_schedule_sequential(const oracle_nodes* nodes, const oracle_pod* pods, int32_t p,
                               const oracle_plugins* pl, int32_t max_pods, int32_t* counts,
                               oracle_result* out);
int oracle_schedule_soa_impl(int32_t n, const uint8_t* unsched, const int8_t* node_digit,
                             int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                             const int32_t* filter_ids, int32_t nf, const int32_t* prescore_ids,
                             int32_t npre, const int32_t* score_ids, const int64_t* weights,
                             const int32_t* norm, int32_t ns, int norm_in_loop, int sequential,
                             int32_t max_pods, int32_t* counts, const int64_t* cols, int32_t* out_idx,
                             int64_t* out_score, int32_t* out_status, uint32_t* out_diag);
/* oracle_schedule_batch_soa with score columns (ORACLE_MAX_COLUMNS x n int64, column k at cols + k*n). */
int oracle_schedule_batch_soa_cols(int32_t n, const uint8_t* unsched, const int8_t* node_digit,
                                   int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                                   const int32_t* filter_ids, int32_t nf, const int32_t* prescore_ids,
                                   int32_t npre, const int32_t* score_ids, const int64_t* weights,
                                   const int32_t* norm, int32_t ns, const int64_t* cols,
                                   int32_t* out_idx, int64_t* out_score, int32_t* out_status);
int oracle_schedule_batch_soa(int32_t n, const uint8_t* unsched, const int8_t* node_digit,
                              int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                              const int32_t* filter_ids, int32_t nf, const int32_t* prescore_ids,
                              int32_t npre, const int32_t* score_ids, const int64_t* weights,
                              const int32_t* norm, int32_t ns, int norm_in_loop,
                              int32_t* out_idx, int64_t* out_score, int32_t* out_status,
                              uint32_t* out_diag);
int oracle_schedule_sequential_soa(int32_t n, const uint8_t* unsched, const int8_t* node_digit,
                                   int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                                   const int32_t* filter_ids, int32_t nf,
                                   const int32_t* prescore_ids, int32_t npre,
                                   const int32_t* score_ids, const int64_t* weights,
                                   const int32_t* norm, int32_t ns, int32_t max_pods,
                                   int32_t* counts, int32_t* out_idx, int64_t* out_score,
                                   int32_t* out_status);
int oracle_suffix_digit(const char* name, int64_t len);

/* Pod-parallel drivers (msh_oracle_omp.c): identical results, pods split over threads. */
int oracle_schedule_batch_soa_cols_omp(int32_t n, const uint8_t* unsched, const int8_t* node_digit,
                                       int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                                       const int32_t* filter_ids, int32_t nf,
                                       const int32_t* prescore_ids, int32_t npre,
                                       const int32_t* score_ids, const int64_t* weights,
                                       const int32_t* norm, int32_t ns, const int64_t* cols,
                                       int32_t threads, int32_t* out_idx, int64_t* out_score,
                                       int32_t* out_status);

#ifdef __cplusplus
}
#endif
#endif
