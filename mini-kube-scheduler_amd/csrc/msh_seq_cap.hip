// msh_seq_cap.hip — the capacity instances of the sequential-commit kernel (msh_seq_kernel.h): one
// workgroup walks the whole batch in order and a commit that fills a node makes it infeasible for the next
// pod (msh_schedule_sequential with max_pods_per_node > 0). A translation unit of its own so that the two
// halves of the kernel family compile in parallel.
#include "msh_seq_kernel.h"

namespace msh {

hipError_t launch_seq_capacity(const SeqArgs& a, int nw, int rs, hipStream_t s) {
  using seqlaunch::launch_seq_nw;
  if (nw == 1) return launch_seq_nw<1, true, 1>(a, rs, 1, s);
  if (nw == 4) return launch_seq_nw<4, true, 1>(a, rs, 1, s);
  return launch_seq_nw<16, true, 1>(a, rs, 1, s);
}

}  // namespace msh
