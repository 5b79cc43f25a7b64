import numpy as np


class boost_ufd:
    """Plain union-find (path halving, link larger root under smaller)."""

    def __init__(self, labels):
        self.parent = np.arange(int(np.max(labels)) + 1 if len(labels) else 0, dtype='int64')

    def _find(self, a):
        p = self.parent
        while p[a] != a:
            p[a] = p[p[a]]
            a = p[a]
        return a

    def merge(self, pairs):
        for a, b in np.asarray(pairs, dtype='int64'):
            ra, rb = self._find(a), self._find(b)
            if ra != rb:
                if ra < rb:
                    self.parent[rb] = ra
                else:
                    self.parent[ra] = rb

    def find(self, labels):
        return np.array([self._find(int(l)) for l in labels], dtype='uint64')
