"""CPU restatement of the reference RelabelWorkflow (TEST INFRASTRUCTURE ONLY; only tests/
import it, the product path is cc_relabel_consecutive in cluster_tools_amd/csrc/cc_relabel.hip).

Follows relabel/find_uniques.py (np.unique per block), relabel/find_labeling.py:84-120 (unique
of the block uniques; new ids arange(start, start + n) with start 0 when uniques[0] == 0, else
1; assignments = [uniques, new_ids]) and the relabel Write (write.py: every voxel's id replaced
through the assignment table).  The block split does not change the result (the union of the
block uniques is the volume's uniques), so it is restated on the whole volume.
"""
import numpy as np


def relabel_consecutive(labels):
    labels = np.asarray(labels, dtype=np.uint64)
    uniques = np.unique(labels)
    start = 0 if uniques.size and uniques[0] == 0 else 1
    new_ids = np.arange(start, start + uniques.size, dtype=np.uint64)
    assignments = np.concatenate([uniques[:, None], new_ids[:, None]], axis=1)
    out = new_ids[np.searchsorted(uniques, labels)]
    return out, assignments
