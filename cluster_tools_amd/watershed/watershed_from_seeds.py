#! /usr/bin/python
"""WatershedFromSeeds task + job (reference: cluster_tools/watershed/watershed_from_seeds.py).

Same task surface as the reference (:20-128): parameters input_path / input_key / seeds_path /
seeds_key / output_path / output_key / mask_path / mask_key / dependency, the task config
(channel_begin, channel_end, agglomerate_channels, size_filter), the uint64 output dataset with
chunks block_shape // 2 clipped to the shape (gzip), and the job's block contract: per block of the
blocking the seeds grow over the normalized input (_ws_block, :143-166), masked blocks without a
mask voxel are skipped and the result is zeroed outside the mask (_ws_block_masked, :169-206).  The
job's compute runs on the MI355X through cc_watershed_from_seeds, one GPU job for the volume.

The reference's watershed call (`vu.watershed`) does not exist in its volume_utils; the watershed
here is defined in include/cc_mi355x.h (minimax path cost from the seeds, smallest label among the
optimal predecessors, 6-connected inside each block) -- parity unpinned.  4-D (channel) input
follows the reference's _read_data (:127-139): the channels channel_begin:channel_end of each block
are normalized together (one min / max over the 4-D block) and aggregated by np.mean / max / min
over the channels (cc_normalize_channels, pinned by goldens made from the reference's own
_read_data: tests/golden/make_golden_ws_read.py); the watershed then takes those values as its
(already normalized) input.  Not supported (raise): size_filter > 0.
"""
import json
import os

import numpy as np

from cluster_tools_amd.luigi_compat import Task, Parameter, TaskParameter
from cluster_tools_amd.cluster_tasks import LocalTask, DummyTask
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu


class WatershedFromSeedsBase(Task):
    task_name = 'watershed_from_seeds'
    src_file = os.path.abspath(__file__)

    input_path = Parameter()
    input_key = Parameter()
    seeds_path = Parameter()
    seeds_key = Parameter()
    output_path = Parameter()
    output_key = Parameter()
    mask_path = Parameter(default='')
    mask_key = Parameter(default='')
    dependency = TaskParameter(default=DummyTask())

    def requires(self):
        return self.dependency

    @staticmethod
    def default_task_config():
        config = LocalTask.default_task_config()
        config.update({'channel_begin': 0, 'channel_end': None,
                       'agglomerate_channels': 'mean', 'size_filter': 0})
        return config

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        if len(shape) == 4:                           # channels first (watershed_from_seeds.py:219-220)
            shape = shape[1:]
        config = self.get_task_config()
        assert config.get('agglomerate_channels', 'mean') in ('mean', 'max', 'min')
        if config.get('size_filter', 0):
            raise NotImplementedError('size_filter > 0 is not supported (the reference watershed is undefined)')
        chunks = tuple(bs // 2 for bs in block_shape)
        chunks = tuple(max(1, min(ch, sh)) for ch, sh in zip(chunks, shape))
        with vu.file_reader(self.output_path) as f:
            f.require_dataset(self.output_key, shape=shape, chunks=chunks, compression='gzip', dtype='uint64')
        config.update({'input_path': self.input_path, 'input_key': self.input_key,
                       'seeds_path': self.seeds_path, 'seeds_key': self.seeds_key,
                       'output_path': self.output_path, 'output_key': self.output_key,
                       'block_shape': block_shape})
        if self.mask_path != '':
            assert self.mask_key != ''
            config.update({'mask_path': self.mask_path, 'mask_key': self.mask_key})
        block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end)
        self._write_log('scheduling %i blocks to be processed' % len(block_list))
        n_jobs = 1                     # one GPU job grows the whole volume
        self.prepare_jobs(n_jobs, block_list, config)
        self.submit_jobs(n_jobs)
        self.wait_for_jobs()
        self.check_jobs(n_jobs)


class WatershedFromSeedsLocal(WatershedFromSeedsBase, LocalTask):
    pass


def _blocks_box(shape, block_shape, block_list):
    """The block-aligned bounding box of the listed blocks: blocks are independent (no halo), so
    the watershed of the box's blocks equals theirs in the whole volume (the box starts on block
    faces, so its own blocking is the volume's)."""
    blocking = vu.Blocking([0, 0, 0], shape, block_shape)
    beg, end = list(shape), [0, 0, 0]
    for b in block_list:
        bl = blocking.getBlock(b)
        beg = [min(p, q) for p, q in zip(beg, bl.begin)]
        end = [max(p, q) for p, q in zip(end, bl.end)]
    return blocking, [(b, e) for b, e in zip(beg, end)]


def watershed_from_seeds(job_id, config_path):
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.thresholded_components.block_components import _read, read_mask, device_mask
    fu.log('start processing job %i' % job_id)
    fu.log('reading config from %s' % config_path)
    with open(config_path) as f:
        config = json.load(f)
    block_list = config['block_list']
    block_shape = config['block_shape']
    shape = list(vu.get_shape(config['input_path'], config['input_key']))
    four_d = len(shape) == 4
    if four_d:
        shape = shape[1:]
    if not block_list:
        fu.log_job_success(job_id)
        return
    # only the listed blocks' bounding box is read and grown (not the whole volume)
    blocking, box = _blocks_box(shape, block_shape, block_list)
    bshape = [e - b for b, e in box]
    if four_d:
        # _read_data (watershed_from_seeds.py:127-139): channels channel_begin:channel_end
        n_ch = vu.get_shape(config['input_path'], config['input_key'])[0]
        c0, c1, _ = slice(config.get('channel_begin', 0), config.get('channel_end', None)).indices(n_ch)
        if c1 <= c0:
            raise ValueError('empty channel range %s:%s' % (config.get('channel_begin', 0), config.get('channel_end')))
        x = _read(config['input_path'], config['input_key'], box=[(c0, c1)] + box,
                  dtype=np.float32)                   # normalize's astype('float32')
    else:
        x = _read(config['input_path'], config['input_key'], box=box, dtype=np.float32)
    seeds = _read(config['seeds_path'], config['seeds_key'], box=box, dtype=np.uint64)
    mask, resized = read_mask(config, shape, box)
    device = int(os.environ.get('CC_DEVICE', '0'))
    dev = torch.device('cuda', device)
    torch.cuda.set_device(dev)
    with _lib.Context(device) as ctx:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        md = device_mask(ctx, mask, resized, shape, dev, box[0][0], bshape[0])
        if md is not None and resized:                # rows of the box, the full (Y, X): crop y / x
            md = md[:, box[1][0]:box[1][1], box[2][0]:box[2][1]].contiguous()
        sd = torch.from_numpy(seeds.view(np.int64)).to(dev)
        xd = torch.from_numpy(x).to(dev)
        if four_d:
            xd = ctx.normalize_channels(xd, block_shape, config.get('agglomerate_channels', 'mean'))
        out, rounds = ctx.watershed_from_seeds(xd, sd, block_shape, md, out=sd, prenormalized=four_d)
        out = out.cpu().numpy().view(np.uint64)
        mh = None if md is None else md.cpu().numpy()
    fu.log('watershed: %d relaxation rounds over the box %s' % (rounds, box))
    with vu.file_reader(config['output_path']) as f:
        ds = f[config['output_key']]
        for b in block_list:
            bb = vu.block_to_bb(blocking.getBlock(b))
            lb = tuple(slice(s.start - o[0], s.stop - o[0]) for s, o in zip(bb, box))
            if mh is not None and not mh[lb].any():          # _ws_block_masked: nothing to do
                fu.log_block_success(b)
                continue
            ds[bb] = out[lb]
            fu.log_block_success(b)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    import sys
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    watershed_from_seeds(job_id, path)
