import numpy as np


def relabelConsecutive(labels, start_label=1, keep_zeros=True, out=None):
    # the reference discards this result (merge_assignments.py:131, typo'd name)
    uniq, inv = np.unique(labels, return_inverse=True)
    return inv.astype(labels.dtype), int(len(uniq)), None
