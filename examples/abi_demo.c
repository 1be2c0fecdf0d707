/* Plain-C consumer of libminisched_hip.so: the calls a cgo binding makes,
 * with no Python, PyTorch or HIP headers in between.
 *
 * It replays the reference's scenario (sched.go:70-143): nine unschedulable nodes node0..node8
 * and pod1 -> FitError; node10 added -> pod1 placed on node10. Names go through the native
 * packer (msh_pack_nodes / msh_pack_pods: List order, suffix digits, tolerations), the batch
 * through msh_schedule_batch. Exit status: 0 = the known answer, 3 = no GPU (MSH_ERR_NO_DEVICE,
 * reported, not a fallback), anything else = failure. One JSON line on stdout.
 *
 * Build (done by mini-kube-scheduler_amd/build.py):
 *   gcc -std=c11 -Iinclude examples/abi_demo.c -Lmini-kube-scheduler_amd -lminisched_hip
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "minisched_hip.h"

#define MAXN 16

static int pack_names(const char* const* names, int n, char* blob, int64_t* off) {
  off[0] = 0;
  for (int i = 0; i < n; ++i) {
    const size_t len = strlen(names[i]);
    memcpy(blob + off[i], names[i], len);
    off[i + 1] = off[i] + (int64_t)len;
  }
  return 0;
}

/* One scheduling cycle of pod1 against `n` nodes; returns the node name index (List order
 * mapped back to the input order) or -1, and the status. */
static int cycle(msh_ctx* ctx, const char* const* node_names, const uint8_t* unsched, int n,
                 int32_t* out_status, int32_t* out_input_idx) {
  char blob[512];
  int64_t off[MAXN + 1];
  int32_t order[MAXN];
  uint8_t u[MAXN];
  int8_t d[MAXN];
  pack_names(node_names, n, blob, off);
  int rc = msh_pack_nodes(n, blob, off, unsched, order, u, d);
  if (rc != MSH_OK) return rc;
  if ((rc = msh_upload_nodes(ctx, n, u, d)) != MSH_OK) return rc;

  const char* pod_names[1] = {"pod1"};
  char pblob[16];
  int64_t poff[2];
  pack_names(pod_names, 1, pblob, poff);
  const int64_t tol_off[2] = {0, 0}; /* pod1 has no tolerations */
  msh_toleration none = {0, 0, 0, 0};
  int8_t pd[1];
  uint8_t pt[1];
  if ((rc = msh_pack_pods(1, pblob, poff, &none, tol_off, pd, pt)) != MSH_OK) return rc;

  int32_t idx[1], st[1];
  int64_t score[1];
  if ((rc = msh_schedule_batch(ctx, 1, pd, pt, idx, score, st)) != MSH_OK) return rc;
  *out_status = st[0];
  *out_input_idx = idx[0] >= 0 ? order[idx[0]] : -1;
  return MSH_OK;
}

int main(void) {
  int ndev = 0;
  msh_device_count(&ndev);
  msh_ctx* ctx = NULL;
  int rc = msh_create(0, &ctx);
  if (rc == MSH_ERR_NO_DEVICE) {
    printf("{\"abi\": %d, \"devices\": %d, \"result\": \"MSH_ERR_NO_DEVICE\"}\n", msh_abi_version(), ndev);
    return 3;
  }
  if (rc != MSH_OK) {
    printf("{\"error\": \"msh_create %d\"}\n", rc);
    return 1;
  }
  const char* names[MAXN] = {"node0", "node1", "node2", "node3", "node4",
                             "node5", "node6", "node7", "node8", "node10"};
  uint8_t unsched[MAXN] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 0};
  int32_t st1 = -1, at1 = -1, st2 = -1, at2 = -1;
  rc = cycle(ctx, names, unsched, 9, &st1, &at1); /* node0..node8, all unschedulable */
  if (rc == MSH_OK) rc = cycle(ctx, names, unsched, 10, &st2, &at2); /* + node10 */
  if (rc != MSH_OK) {
    printf("{\"error\": \"%d: %s\"}\n", rc, msh_last_error(ctx));
    msh_destroy(ctx);
    return 1;
  }
  const int ok = st1 == MSH_FIT_ERROR && at1 == -1 && st2 == MSH_PLACED && at2 == 9;
  printf("{\"abi\": %d, \"devices\": %d, \"phase1\": {\"status\": %d}, \"phase2\": {\"status\": %d, "
         "\"node\": \"%s\"}, \"known_answer\": %s}\n",
         msh_abi_version(), ndev, st1, st2, at2 >= 0 ? names[at2] : "", ok ? "true" : "false");
  msh_destroy(ctx);
  return ok ? 0 : 2;
}
