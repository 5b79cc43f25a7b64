"""The z-slab sharded path's device entry points (cc_shard_*), run for several slabs on one
GPU in one process (distributed.label_slabs_single_process), against the oracle on the
whole volume: raw uint64 labels and the assembled LUT must be identical."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('n_slabs,shape,block_shape,mode', [
    (2, (64, 256, 256), (32, 128, 128), 'greater'),
    (2, (64, 256, 256), (32, 128, 128), 'less'),
    (4, (128, 200, 300), (32, 64, 128), 'less'),
    (3, (75, 130, 170), (25, 64, 64), 'greater'),
    (8, (64, 96, 160), (8, 48, 64), 'less'),
])
def test_sharded_single_gpu_vs_oracle(n_slabs, shape, block_shape, mode):
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    x = O.boundary_map(shape, origin=(3, 0, 9))
    ctxs = [_lib.Context(0) for _ in range(n_slabs)]
    try:
        lab, res, sums, luts = label_slabs_single_process(ctxs, torch.from_numpy(x).cuda(), block_shape, 0.5, mode)
        ref = O.label_volume(x, block_shape, 0.5, mode, n_threads=8)
        np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
        assert sum(sums) + 1 == ref['n_labels']
        np.testing.assert_array_equal(assemble_lut(luts, sums), ref['lut'])
        assert sum(r['n_components'] for r in res) == len(np.unique(ref['labels'])) - 1
    finally:
        for c in ctxs:
            c.close()
