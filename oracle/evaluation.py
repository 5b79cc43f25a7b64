"""CPU restatement of the reference evaluation path (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module; the product path (cc_evaluate in
cluster_tools_amd/csrc/cc_eval.hip) never calls it.

Follows:
  * node_labels/block_node_labels.py:133-166 (_labels_for_block): per block of the block grid,
    skip when ws.sum() == 0; skip when every label equals ignore_label; otherwise
    ndist.computeAndSerializeLabelOverlaps(ws, labs, withIgnoreLabel, ignoreLabel) -- overlaps
    {ws id: {label id: count}} of the voxels whose label is not ignore_label.  MergeNodeLabels
    (node_labels/merge_node_labels.py:121-155, max_overlap=False, serialize_counts=True) sums the
    block overlaps per ws id into chunks of ws ids, so measures.py:120-128 merging the chunk
    dicts by update loses nothing: a (ws, label) pair's count is summed over all blocks.
  * evaluation/measures.py:81-117 (contigency_table_from_overlaps): p_ids = [gt id, ws id],
    a = gt sizes, b = ws sizes, n_points.
  * the measures of elf.evaluation (compute_vi_scores / compute_rand_scores, measures.py:154-155):
    elf is not installed here, so these are restated from their published definitions --
    vi_split = H(seg|gt), vi_merge = H(gt|seg) in bits, adapted rand error 1 - 2PR/(P+R) with
    P = sum p^2 / sum b^2, R = sum p^2 / sum a^2, rand index 1 - (sum a^2 + sum b^2 - 2 sum p^2)/N^2.
    Parity of these formulas with elf is UNPINNED (no elf, no golden vectors for them); the
    contingency table is pinned by construction to the reference's block loop.
"""
import numpy as np


def block_overlaps(seg, gt, block_shape, ignore_label=0):
    """{(seg id, gt id): count} over the block grid (block_node_labels.py:133-166)."""
    seg = np.asarray(seg)
    gt = np.asarray(gt)
    assert seg.shape == gt.shape and seg.ndim == 3
    ov = {}
    nb = [(s + b - 1) // b for s, b in zip(seg.shape, block_shape)]
    for bz in range(nb[0]):
        for by in range(nb[1]):
            for bx in range(nb[2]):
                bb = tuple(slice(i * b, min((i + 1) * b, s))
                           for i, b, s in zip((bz, by, bx), block_shape, seg.shape))
                ws = seg[bb]
                if ws.sum() == 0:                       # :141
                    continue
                labs = gt[bb].astype('uint64')
                if ignore_label is not None:
                    if np.sum(labs == ignore_label) == labs.size:   # :151-155
                        continue
                    keep = labs != ignore_label
                    w, g = ws[keep].astype(np.uint64), labs[keep]
                else:
                    w, g = ws.ravel().astype(np.uint64), labs.ravel()
                if w.size == 0:
                    continue
                pairs, counts = np.unique(np.stack([w, g], axis=1), axis=0, return_counts=True)
                for (a, b), c in zip(pairs.tolist(), counts.tolist()):
                    ov[(a, b)] = ov.get((a, b), 0) + c
    return ov


def contingency_table(ov):
    """measures.py:92-117 on the merged overlaps: (a_dict gt sizes, b_dict seg sizes, p_counts, n)."""
    a_dict, b_dict = {}, {}
    p_counts = np.array([c for c in ov.values()], dtype='float64')
    for (ws_id, gt_id), c in ov.items():
        a_dict[gt_id] = a_dict.get(gt_id, 0) + c
        b_dict[ws_id] = b_dict.get(ws_id, 0) + c
    n_points = int(sum(a_dict.values()))
    assert n_points == sum(b_dict.values()) == int(p_counts.sum())
    return a_dict, b_dict, p_counts, n_points


def measures(seg, gt, block_shape, ignore_label=0):
    """The four numbers of measures.py:157-158 plus the table sizes (cc_eval_result fields)."""
    ov = block_overlaps(seg, gt, block_shape, ignore_label)
    a_dict, b_dict, p_counts, n = contingency_table(ov)
    out = {'n_points': n, 'n_pairs': len(ov), 'n_seg_ids': len(b_dict), 'n_gt_ids': len(a_dict)}
    if n == 0:
        return out, ov
    a = np.array(list(a_dict.values()), dtype='float64')
    b = np.array(list(b_dict.values()), dtype='float64')

    def h(c):
        p = c / n
        return float(-np.sum(p * np.log2(p)))

    h_ab, h_a, h_b = h(p_counts), h(a), h(b)
    sum_a, sum_b, sum_ab = float(np.sum(a * a)), float(np.sum(b * b)), float(np.sum(p_counts * p_counts))
    prec, rec = sum_ab / sum_b, sum_ab / sum_a
    out.update({'vi_split': h_ab - h_a, 'vi_merge': h_ab - h_b,
                'adapted_rand_error': 1.0 - 2.0 * prec * rec / (prec + rec),
                'rand_index': 1.0 - (sum_a + sum_b - 2.0 * sum_ab) / float(n) ** 2})
    return out, ov
