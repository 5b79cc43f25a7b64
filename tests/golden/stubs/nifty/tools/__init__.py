import numpy as np


class _Block:
    def __init__(self, begin, end):
        self.begin = list(begin)
        self.end = list(end)
        self.shape = [e - b for b, e in zip(begin, end)]


class blocking:
    def __init__(self, roiBegin, roiEnd, blockShape):
        self.roiBegin = list(roiBegin)
        self.roiEnd = list(roiEnd)
        self.blockShape = list(blockShape)
        self.blocksPerAxis = [-(-(e - b) // s) for b, e, s in zip(self.roiBegin, self.roiEnd, self.blockShape)]
        self.numberOfBlocks = int(np.prod(self.blocksPerAxis))

    def _coord(self, block_id):
        return list(np.unravel_index(block_id, self.blocksPerAxis))

    def getBlock(self, blockIndex):
        c = self._coord(blockIndex)
        begin = [rb + ci * s for rb, ci, s in zip(self.roiBegin, c, self.blockShape)]
        end = [min(b + s, re) for b, s, re in zip(begin, self.blockShape, self.roiEnd)]
        return _Block(begin, end)

    def getNeighborId(self, blockId, axis, lower):
        c = self._coord(blockId)
        c[axis] += -1 if lower else 1
        if c[axis] < 0 or c[axis] >= self.blocksPerAxis[axis]:
            return -1
        return int(np.ravel_multi_index(c, self.blocksPerAxis))


def take(relabeling, toRelabel):
    return np.asarray(relabeling)[toRelabel]


def takeDict(relabeling, toRelabel):
    return np.vectorize(lambda v: relabeling[v], otypes=[toRelabel.dtype])(toRelabel)
