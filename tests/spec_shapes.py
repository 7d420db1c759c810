"""Dataset shapes (sites, taxa, hard sites, block_threads) of the GPU tests -- TEST INFRASTRUCTURE.

__graft_entry__.build() compiles their shape-specialised sweep kernels into the in-tree cache (sr_specialize
needs only the shape; no GPU) so that the GPU suite loads them instead of compiling ~4 s per new shape on the
box.  A shape missing here is still compiled at session creation -- the list only saves time."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def shapes():
    sys.path.insert(0, HERE)
    import test_gpu_edge
    import test_gpu_jit
    import test_gpu_fuzz
    out = {(N, M, nh, tb) for _, N, M, nh, tb in test_gpu_edge.CASES}
    out |= set(test_gpu_fuzz.lds_shapes())
    out |= {(spec[0], spec[1], spec[2], 0) for _, spec, _ in test_gpu_jit.CASES if spec is not None}
    out |= {(256, 300, 5, 0), (400, 150, 5, 0),   # test_gpu_edge.test_steep_walks
            (70, 90, 3, 0), (70, 90, 9, 0),      # test_gpu_jit shards, test_gpu_multi
            (40, 24, 3, 0)}                      # test_gpu_edge.test_johnk_beta_branch
    return sorted(out)
