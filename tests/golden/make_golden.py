#!/opt/conda/bin/python3.9
"""Generate golden vectors by running the REFERENCE's own hot-path job functions.

Run only in the build container (it needs /root/reference and the conda python
with scikit-image 0.18.3):

    /opt/conda/bin/python3.9 tests/golden/make_golden.py

What runs: the reference's job functions, unmodified, imported from
/root/reference with small local stand-ins for the absent dependencies
(tests/golden/stubs: luigi, nifty, vigra, elf; storage is h5py instead of z5py):

    block_components   cluster_tools/thresholded_components/block_components.py:236
    merge_offsets      cluster_tools/thresholded_components/merge_offsets.py:83
    block_faces        cluster_tools/thresholded_components/block_faces.py:140
    merge_assignments  cluster_tools/thresholded_components/merge_assignments.py:88
    write              cluster_tools/write/write.py:292

driven with hand-written job configs exactly as LocalTask.prepare_jobs would
write them (cluster_tools/cluster_tasks.py:301-335: block_list[job_id::n_jobs]).

Real arithmetic kept: the reference's normalize / threshold / mask / offset / face
/ write code with numpy 1.26.4 and skimage 0.18.3 `label`.  Stubbed: the union-find
(representative choice differs from nifty's boost_ufd; the partition does not).

Output: tests/golden/<case>.npz (plain arrays, allow_pickle=False safe) plus
tests/golden/index.json.  Labels are stored canonically relabelled (first
occurrence in C order); the block-local labels of stage 1 are stored RAW (they
are skimage's own numbering, pinned by 0.18.3).
"""
import json
import os
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, os.path.join(HERE, 'stubs'))
sys.path.insert(0, REPO)


def _bare_package(name, path):
    mod = types.ModuleType(name)
    mod.__path__ = [path]
    sys.modules[name] = mod
    return mod


# bypass the eager package __init__ imports (cluster_tools/__init__.py:1-5)
_bare_package('cluster_tools', os.path.join(REF, 'cluster_tools'))
_bare_package('cluster_tools.utils', os.path.join(REF, 'cluster_tools', 'utils'))
_bare_package('cluster_tools.thresholded_components',
              os.path.join(REF, 'cluster_tools', 'thresholded_components'))
_bare_package('cluster_tools.write', os.path.join(REF, 'cluster_tools', 'write'))

import h5py  # noqa: E402
from cluster_tools.thresholded_components import block_components as ref_bc  # noqa: E402
from cluster_tools.thresholded_components import merge_offsets as ref_mo  # noqa: E402
from cluster_tools.thresholded_components import block_faces as ref_bf  # noqa: E402
from cluster_tools.thresholded_components import merge_assignments as ref_ma  # noqa: E402
from cluster_tools.write import write as ref_wr  # noqa: E402
from oracle.synth import boundary_q, ellipsoid_mask  # noqa: E402


def canon(labels):
    """First-occurrence (C order) consecutive relabel; 0 stays 0."""
    flat = np.asarray(labels).ravel()
    out = np.zeros(flat.shape, dtype=np.uint32)
    nz = flat != 0
    if nz.any():
        vals = flat[nz]
        uniq, first, inv = np.unique(vals, return_index=True, return_inverse=True)
        order = np.argsort(first, kind='stable')
        rank = np.empty(len(uniq), dtype=np.uint32)
        rank[order] = np.arange(1, len(uniq) + 1, dtype=np.uint32)
        out[nz] = rank[inv]
    return out.reshape(np.shape(labels))


def n_blocks_of(shape, block_shape):
    return int(np.prod([-(-s // b) for s, b in zip(shape, block_shape)]))


def run_reference(inp, block_shape, threshold, mode, mask=None, n_jobs_bc=2, n_jobs_bf=1, channel=None, extra=None,
                  compression='gzip'):
    """Run the five reference stages in a scratch folder; return artefacts.  channel (int or
    list): inp is 4-D (C, Z, Y, X) and block_components averages those channels
    (block_components.py:150-159).  compression None: an uncompressed scratch output (large
    cases; the storage codec does not enter the arithmetic)."""
    tmp = tempfile.mkdtemp(prefix='golden_')
    try:
        in_path = os.path.join(tmp, 'in.h5')
        out_path = os.path.join(tmp, 'out.h5')
        with h5py.File(in_path, 'w') as f:
            f.create_dataset('raw', data=inp)
            if mask is not None:
                f.create_dataset('mask', data=mask)
        shape = inp.shape if channel is None else inp.shape[1:]
        # output dataset as BlockComponentsBase.run_impl creates it (block_components.py:99-106)
        chunks = tuple(max(1, min(bs // 2, sh)) for bs, sh in zip(block_shape, shape))
        with h5py.File(out_path, 'w') as f:
            f.require_dataset('seg', shape=shape, dtype='uint64', compression=compression, chunks=chunks)
        nb = n_blocks_of(shape, block_shape)
        block_list = list(range(nb))

        def job_cfgs(name, n_jobs, cfg):
            paths = []
            for j in range(n_jobs):
                c = dict(cfg)
                c['block_list'] = block_list[j::n_jobs]
                p = os.path.join(tmp, '%s_job_%i.config' % (name, j))
                with open(p, 'w') as fh:
                    json.dump(c, fh)
                paths.append(p)
            return paths

        n_bc = min(nb, n_jobs_bc)
        cfg = {'input_path': in_path, 'input_key': 'raw', 'output_path': out_path,
               'output_key': 'seg', 'block_shape': list(block_shape), 'tmp_folder': tmp,
               'threshold': float(threshold), 'threshold_mode': mode}
        if mask is not None:
            cfg.update({'mask_path': in_path, 'mask_key': 'mask'})
        if channel is not None:
            cfg['channel'] = channel
        cfg.update(extra or {})          # e.g. sigma_prefilter (make_golden_sigma.py)
        for j, p in enumerate(job_cfgs('block_components', n_bc, cfg)):
            ref_bc.block_components(j, p)
        # per-block values v_i (n_i + 1 or 0) before merge_offsets deletes the files
        vals = {}
        for j in range(n_bc):
            with open(os.path.join(tmp, 'connected_components_offsets_%i.json' % j)) as fh:
                vals.update({int(k): int(v) for k, v in json.load(fh).items()})
        block_values = np.array([vals[b] for b in range(nb)], dtype=np.uint64)
        with h5py.File(out_path, 'r') as f:
            local_labels = f['seg'][:]

        offsets_path = os.path.join(tmp, 'cc_offsets.json')
        p = os.path.join(tmp, 'merge_offsets_job_0.config')
        with open(p, 'w') as fh:
            json.dump({'tmp_folder': tmp, 'n_jobs': n_bc, 'save_path': offsets_path,
                       'n_blocks': nb, 'save_prefix': 'connected_components_offsets'}, fh)
        ref_mo.merge_offsets(0, p)
        with open(offsets_path) as fh:
            off = json.load(fh)

        n_bf = min(nb, n_jobs_bf)
        for j, p in enumerate(job_cfgs('block_faces', n_bf, {
                'input_path': out_path, 'input_key': 'seg', 'offsets_path': offsets_path,
                'block_shape': list(block_shape), 'tmp_folder': tmp})):
            ref_bf.block_faces(j, p)
        pairs = [np.load(os.path.join(tmp, 'cc_assignments_%i.npy' % j)) for j in range(n_bf)]
        pairs = [pp.reshape(-1, 2).astype(np.uint64) for pp in pairs if pp.size]
        pairs = (np.unique(np.concatenate(pairs, axis=0), axis=0) if pairs
                 else np.zeros((0, 2), dtype=np.uint64))

        p = os.path.join(tmp, 'merge_assignments_job_0.config')
        with open(p, 'w') as fh:
            json.dump({'output_path': out_path, 'output_key': 'assignments', 'tmp_folder': tmp,
                       'n_jobs': n_bf, 'offset_path': offsets_path,
                       'save_prefix': 'cc_assignments'}, fh)
        ref_ma.merge_assignments(0, p)
        with h5py.File(out_path, 'r') as f:
            lut = f['assignments'][:]

        n_wr = min(nb, 2)
        for j, p in enumerate(job_cfgs('write', n_wr, {
                'input_path': out_path, 'input_key': 'seg', 'block_shape': list(block_shape),
                'assignment_path': out_path, 'assignment_key': 'assignments',
                'offset_path': offsets_path, 'threads_per_job': 1,
                'allow_empty_assignments': False})):
            ref_wr.write(j, p)
        with h5py.File(out_path, 'r') as f:
            labels = f['seg'][:]
            max_id = int(f['seg'].attrs['maxId'])
        return dict(block_values=block_values, local_labels=local_labels,
                    offsets=np.array(off['offsets'], dtype=np.uint64),
                    empty_blocks=np.array(off['empty_blocks'], dtype=np.int64),
                    n_labels=int(off['n_labels']), pairs=pairs, lut=lut,
                    labels=labels, max_id=max_id)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def make_cases():
    rng = np.random.default_rng(20240611)
    cases = []

    def add(name, inp, block_shape, threshold, mode, mask=None, store_q=None, **kw):
        cases.append(dict(name=name, inp=inp, block_shape=block_shape, threshold=threshold,
                          mode=mode, mask=mask, store_q=store_q, kw=kw))

    # synthetic boundary maps (stored as uint8 q; value = q / 256 exactly)
    shp = (40, 72, 88)
    q = boundary_q(shp)
    bm = q.astype(np.float32) / np.float32(256)
    add('bmap_greater', bm, (16, 32, 32), 0.5, 'greater', store_q=q)
    add('bmap_less', bm, (16, 32, 32), 0.5, 'less', store_q=q)
    add('bmap_equal0', bm, (16, 32, 32), 0.0, 'equal', store_q=q)
    add('bmap_equal_half', bm, (16, 32, 32), 0.5, 'equal', store_q=q)
    add('bmap_greater_t03', bm, (16, 32, 32), 0.3, 'greater', store_q=q)
    add('bmap_mask', bm, (16, 32, 32), 0.5, 'greater', mask=ellipsoid_mask(shp), store_q=q)
    add('bmap_mask_less', bm, (16, 32, 32), 0.5, 'less', mask=ellipsoid_mask(shp, 0.3), store_q=q)
    add('bmap_odd_blocks', bm, (5, 7, 9), 0.5, 'greater', store_q=q)
    add('bmap_one_block', bm, (64, 128, 128), 0.5, 'greater', store_q=q)
    add('bmap_flat_blocks', bm, (2, 72, 88), 0.5, 'less', store_q=q)
    add('bmap_quirk', bm, (16, 32, 32), 0.5, 'greater', store_q=q, n_jobs_bf=10 ** 6)
    q2 = boundary_q((48, 96, 96), origin=(100, 37, 0))
    add('bmap_big', q2.astype(np.float32) / np.float32(256), (32, 64, 64), 0.5, 'greater', store_q=q2)
    add('bmap_big_less', q2.astype(np.float32) / np.float32(256), (32, 64, 64), 0.5, 'less', store_q=q2)

    # white noise: many tiny components, every 26-neighbour case occurs
    wn = rng.random((12, 18, 24), dtype=np.float32)
    add('noise_tiny_blocks', wn, (4, 6, 8), 0.7, 'greater')
    add('noise_less', wn, (4, 6, 8), 0.25, 'less')
    add('noise_t01', wn, (6, 9, 12), 0.1, 'less')

    # normalisation edge cases: per-block affine rescaling, constant block, NaN block, inf
    sm = rng.random((16, 24, 32), dtype=np.float32)
    sm[:8, :12, :16] = sm[:8, :12, :16] * np.float32(1000.0) + np.float32(5.0)
    sm[8:, 12:, 16:] = sm[8:, 12:, 16:] * np.float32(1e-3) - np.float32(7.0)
    sm[:8, 12:, :16] = np.float32(0.3)          # constant block: mx == 0, no division
    sm[8:, :12, 16:] = np.float32(np.nan)       # NaN block: no foreground
    sm[8:, :12, :16] *= np.float32(3.0)
    sm[9, 3, 5] = np.float32(np.nan)            # lone NaN poisons its block
    add('norm_edge_greater', sm, (8, 12, 16), 0.5, 'greater')
    add('norm_edge_less', sm, (8, 12, 16), 0.5, 'less')
    add('norm_edge_equal0', sm, (8, 12, 16), 0.0, 'equal')
    inf = rng.random((8, 12, 16), dtype=np.float32)
    inf[0, 0, 0] = np.float32(np.inf)
    inf[4, 6, 8] = np.float32(-np.inf)
    add('inf_block', inf, (4, 12, 16), 0.4, 'less')
    # denormals and tiny ranges
    dn = (rng.random((8, 12, 16), dtype=np.float32) * np.float32(1e-38)).astype(np.float32)
    add('denormal_range', dn, (4, 6, 8), 0.5, 'greater')
    # integer levels: 'equal' hits normalised 0.5 exactly; mask values other than 0/1
    lv = rng.integers(0, 3, size=(12, 18, 24)).astype(np.float32)
    mk = rng.choice(np.array([0, 7, 255], dtype=np.uint8), size=(12, 18, 24), p=[0.2, 0.4, 0.4])
    add('levels_equal_half', lv, (4, 6, 8), 0.5, 'equal')
    add('levels_equal_half_mask', lv, (4, 6, 8), 0.5, 'equal', mask=mk)
    # all background and all foreground
    add('all_zero', np.zeros((8, 12, 16), np.float32), (4, 6, 8), 0.5, 'greater')
    add('all_fg_const', np.zeros((8, 12, 16), np.float32), (4, 6, 8), 0.5, 'less')
    return cases


def main():
    out_dir = HERE
    index = {}
    for case in make_cases():
        kw = dict(case['kw'])
        n_jobs_bf = kw.pop('n_jobs_bf', 1)
        res = run_reference(case['inp'], case['block_shape'], case['threshold'], case['mode'],
                            mask=case['mask'], n_jobs_bf=n_jobs_bf)
        arrays = dict(
            block_shape=np.array(case['block_shape'], dtype=np.int64),
            threshold=np.array(case['threshold'], dtype=np.float64),
            block_values=res['block_values'], offsets=res['offsets'],
            empty_blocks=res['empty_blocks'], n_labels=np.array(res['n_labels'], dtype=np.uint64),
            local_labels=res['local_labels'].astype(np.uint32),
            pairs=res['pairs'],
            lut_canon=canon(res['lut']),
            labels_canon=canon(res['labels']),
            max_id=np.array(res['max_id'], dtype=np.uint64))
        assert int(res['local_labels'].max()) < 2 ** 32
        if case['store_q'] is not None:
            arrays['input_q'] = case['store_q']
        else:
            arrays['input'] = case['inp']
        if case['mask'] is not None:
            arrays['mask'] = case['mask']
        np.savez_compressed(os.path.join(out_dir, case['name'] + '.npz'), **arrays)
        n_comp = int(arrays['labels_canon'].max())
        index[case['name']] = dict(shape=list(case['inp'].shape), block_shape=list(case['block_shape']),
                                   threshold=case['threshold'], mode=case['mode'],
                                   mask=case['mask'] is not None,
                                   quirk=n_jobs_bf > 1, n_jobs_block_faces=min(
                                       n_jobs_bf, n_blocks_of(case['inp'].shape, case['block_shape'])),
                                   n_components=n_comp, n_pairs=int(len(res['pairs'])),
                                   n_labels=res['n_labels'])
        print(case['name'], index[case['name']])
    with open(os.path.join(out_dir, 'index.json'), 'w') as fh:
        json.dump(index, fh, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
