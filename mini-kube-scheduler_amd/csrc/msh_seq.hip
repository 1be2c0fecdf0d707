// msh_seq.hip — launchers of the sequential-commit kernel (msh_seq_kernel.h) without a capacity, the
// count fold, and the dispatch of msh_schedule_sequential_device (the capacity instances are in
// msh_seq_cap.hip).
#include "msh_seq_kernel.h"

namespace msh {

using seqlaunch::launch_seq_nw;

// Scanning waves: as few as keep at most 4 words per lane (one wave up to 8,192 nodes, four up to
// 32,768), then 15 (+ the finalizer) waves with up to 12 words per lane without a capacity
// (368,640 nodes; 6 x 12 plane VGPRs per lane), 16 waves with up to 8 with one (262,144 nodes; the
// FULL plane makes 7 per word, and 12 words spill). Per-pod latency is one wave's scan plus one DPP
// reduction; extra waves add an LDS exchange and a barrier.
namespace {
int seq_waves_for(const SeqArgs& a, const DeviceInfo& dev) {
  const bool cap = a.max_pods > 0;
  const int nw_big = cap ? 16 : 15;
  auto rs_for = [&](int nw) { return (a.n_words + nw * WAVE - 1) / (nw * WAVE); };
  // one wave holds up to 4 words per lane (8,192 nodes), 16 with a capacity (32,768: seq_capu_kernel, whose
  // one wave outruns the 4- and 16-wave forms, profiles/ab/r6_seq_waves.txt)
  const int rs1 = cap ? 16 : 4;
  int nw = dev.seq_waves > 0 ? dev.seq_waves : (rs_for(1) <= rs1 ? 1 : rs_for(4) <= 4 ? 4 : nw_big);
  if (nw != 1 && nw != 4) nw = nw_big;
  if (rs_for(nw) > (nw == nw_big ? (cap ? 8 : 12) : nw == 1 ? rs1 : 4)) nw = nw_big;  // an override too small for the table
  return nw;
}

__global__ void count_fold_kernel(int32_t* counts, int64_t stride, int32_t replicas, int32_t n) {
  const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  int32_t sum = counts[i];
  for (int k = 1; k < replicas; ++k) {
    sum += counts[k * stride + i];
    counts[k * stride + i] = 0;
  }
  counts[i] = sum;
}
}  // namespace

hipError_t launch_count_fold(int32_t* counts, int64_t stride, int32_t replicas, int32_t n, hipStream_t s) {
  if (n <= 0 || replicas <= 1) return hipSuccess;
  count_fold_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s>>>(counts, stride, replicas, n);
  return hipGetLastError();
}

// Pod waves per pod-block workgroup (one scanning wave): msh_options.seq_pod_waves, else SEQ_POD_WAVES.
int seq_pod_waves(const DeviceInfo& dev) { return dev.seq_pod_waves > 0 ? dev.seq_pod_waves : SEQ_POD_WAVES; }

// Tables whose counts fit LDS only (up to four scanning waves, 32,768 nodes): a larger table's blocks
// would have no LDS to count in.
int32_t seq_blocks(const SeqArgs& a, const DeviceInfo& dev) {
  if (a.max_pods > 0 || !dev.seq_split || a.n_pods <= WAVE || a.count_replicas < SEQ_COUNT_REPLICAS ||
      seq_waves_for(a, dev) > 4)
    return 1;
  return (a.n_pods + WAVE - 1) / WAVE;
}

hipError_t launch_sequential(const SeqArgs& a, const DeviceInfo& dev, hipStream_t s, std::string* err) {
  if (a.n_pods == 0) return hipSuccess;
  const bool cap = a.max_pods > 0;
  const int nw_big = cap ? 16 : 15;
  const int rs_max = cap ? 8 : 12;
  const int nw = seq_waves_for(a, dev);
  const int rs = (a.n_words + nw * WAVE - 1) / (nw * WAVE);
  // words per lane each form holds: one wave 16 with a capacity (seq_capu_kernel) and 4 without, four
  // waves 4, the big form rs_max (seq_waves_for only picks a form the table fits, the big one last)
  if (rs > (nw == 1 ? (cap ? 16 : 4) : nw == 4 ? 4 : rs_max)) {
    if (err)
      *err = "sequential mode keeps the node table in registers: at most " +
             std::to_string(nw_big * WAVE * rs_max * 32) + " nodes per device" + (cap ? " with a capacity" : "");
    return hipErrorInvalidValue;
  }
  SeqArgs ka = a;
  ka.pods_per_block = a.n_pods;
  if (cap) return launch_seq_capacity(ka, nw, rs, s);
  // Without a capacity: 64-pod blocks of consecutive pods, each one workgroup walking its pods in
  // order (msh_options.seq_split = 1: one workgroup for the whole batch); with one scanning wave (tables
  // up to 8,192 nodes) a block's 64 pods are shared by seq_pod_waves waves that each hold the whole table
  // and walk a sub-block of 64 / seq_pod_waves consecutive pods in order
  const int32_t blocks = seq_blocks(a, dev);
  if (blocks > 1) ka.pods_per_block = WAVE;
  if (nw == 1) {
    switch (blocks > 1 ? seq_pod_waves(dev) : 1) {
      case 2: return launch_seq_nw<1, false, 2>(ka, rs, blocks, s);
      case 4: return launch_seq_nw<1, false, 4>(ka, rs, blocks, s);
      case 8: return launch_seq_nw<1, false, 8>(ka, rs, blocks, s);
      default: return launch_seq_nw<1, false, 1>(ka, rs, blocks, s);
    }
  }
  if (nw == 4) return launch_seq_nw<4, false, 1>(ka, rs, blocks, s);
  return launch_seq_nw<15, false, 1>(ka, rs, blocks, s);
}

}  // namespace msh
