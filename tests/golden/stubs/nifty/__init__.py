"""Stand-in for nifty (absent here): blocking, take and a union-find.

Restated from nifty's documented behaviour (C-order block grid rooted at roiBegin,
edge blocks truncated; getNeighborId(id, axis, lower) -> -1 outside the grid).
The union-find representative choice differs from boost::disjoint_sets; the
partition does not.
"""
