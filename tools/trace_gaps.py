"""Per-kernel busy time and idle gaps of the last step of a rocprofv3 kernel trace (tools/
gpu_steps.sh trace_slabs8: tools/bench_sharded_slabs.py under --kernel-trace).

    python tools/trace_gaps.py TRACE_DIR_OR_CSV [n_slabs]

The last step starts at the n_slabs-th last k_sample (k_clear_front in builds before it was folded
into k_sample; one per slab, the slabs of a step run phase by phase).  For every kernel: launches, summed duration, and the idle time between the
previous kernel's end and its start ("gap-before": host synchronisations, launch latency).
"""
import collections
import csv
import glob
import os
import sys


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True)[0]
    nsl = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    name = [r['Kernel_Name'].split('(')[0].replace('void ', '').replace('cc::', '') for r in rows]
    mark = 'k_clear_front' if any(n.startswith('k_clear_front') for n in name) else 'k_sample'
    first = [i for i, n in enumerate(name) if n.startswith(mark)][-nsl]
    seg = list(zip(name[first:], rows[first:]))
    t0 = int(seg[0][1]['Start_Timestamp'])
    t1 = max(int(r['End_Timestamp']) for _, r in seg)
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for _, r in seg)
    print('last step of %d slabs: span %.3f ms, kernel busy %.3f ms, launches %d'
          % (nsl, (t1 - t0) / 1e6, busy / 1e6, len(seg)))
    acc = collections.defaultdict(lambda: [0, 0])
    gaps = collections.defaultdict(float)
    prev_end = None
    for n, r in seg:
        n = n[:40]
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        acc[n][0] += 1
        acc[n][1] += e - s
        if prev_end is not None and s > prev_end:
            gaps[n] += s - prev_end
        prev_end = max(prev_end or 0, e)
    for n, (c, d) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        print('%-42s %3d  %8.4f ms  gap-before %8.4f ms' % (n, c, d / 1e6, gaps[n] / 1e6))
    print('total gaps %.3f ms' % (sum(gaps.values()) / 1e6))


if __name__ == '__main__':
    main()
