"""Summarise rocprofv3 CSV output into per-kernel JSON (used for profiles/ and bench.py's
roofline.traffic).

    python tools/prof_summary.py --trace DIR_WITH_kernel_trace.csv \
        [--fetch DIR_WITH_counter_collection.csv] [--write DIR_...] -o out.json

Per kernel: dispatch count, average duration (from the kernel trace), and per-dispatch HBM
bytes from the PMC passes, corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a coalesced streaming read
of full 128-B lines (16 B / lane per the guide; the 4 B / lane, 256 B per wave-instruction f32
rows of k_spec / k_pass2 read the same way: 9.1 GB raw for the 17.2 GB input), so those are
doubled ('fetch_bytes'); 'fetch_bytes_raw' keeps the uncorrected figure.  Byte-wide reads (the
uint8 mask, 64 B per wave-instruction) are counted exactly (raw k_spec<true> = 8.6 GB f32 / 2 +
4.3 GB mask), so `--narrow KERNEL=BYTES` names the per-dispatch bytes of such reads: they are
taken out of the raw figure before doubling and added back once.  WRITE_SIZE is exact for
16-B-per-lane streaming stores.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def _find(d, pat):
    hits = sorted(glob.glob(os.path.join(d, '**', pat), recursive=True))
    if not hits:
        raise SystemExit('no %s under %s' % (pat, d))
    return hits[-1]


def short(name):
    n = re.sub(r'\(.*$', '', name)            # drop the argument list
    n = re.sub(r'^void ', '', n)
    n = n.replace('cc::', '')
    return n.strip()


def trace_stats(d):
    acc = collections.OrderedDict()
    with open(_find(d, '*kernel_trace.csv')) as f:
        for r in csv.DictReader(f):
            k = short(r['Kernel_Name'])
            ns = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            a = acc.setdefault(k, [0, 0])
            a[0] += 1
            a[1] += ns
    return {k: {'count': c, 'avg_ms': t / c / 1e6, 'total_ms': t / 1e6} for k, (c, t) in acc.items()}


def counter(d, name):
    acc = collections.defaultdict(lambda: [0, 0.0])
    with open(_find(d, '*counter_collection.csv')) as f:
        for r in csv.DictReader(f):
            if r['Counter_Name'] != name:
                continue
            k = short(r['Kernel_Name'])
            acc[k][0] += 1
            acc[k][1] += float(r['Counter_Value'])
    return {k: v / c for k, (c, v) in acc.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--trace', required=True)
    p.add_argument('--fetch')
    p.add_argument('--write')
    p.add_argument('-o', '--out', required=True)
    p.add_argument('--narrow', action='append', default=[],
                   help='KERNEL_PREFIX=BYTES: per-dispatch bytes of byte-wide reads (counted exactly)')
    p.add_argument('--bench-json', default=None,
                   help="the bench line of the profiled run: its lib.src (the library's source hash) and "
                        "workload are stamped into the summary's '_meta', so bench.py uses the traffic "
                        "figures only for the library they were measured on")
    a = p.parse_args()
    narrow = {k: float(v) for k, v in (n.split('=') for n in a.narrow)}
    res = trace_stats(a.trace)
    fetch = counter(a.fetch, 'FETCH_SIZE') if a.fetch else {}
    write = counter(a.write, 'WRITE_SIZE') if a.write else {}
    for k, v in res.items():
        if k in fetch:
            raw = fetch[k] * 1024
            nb = next((b for pre, b in narrow.items() if k.startswith(pre)), 0.0)
            nb = min(nb, raw)
            v['fetch_bytes_raw'] = raw
            v['fetch_bytes'] = 2 * (raw - nb) + nb
            if nb:
                v['fetch_narrow_bytes'] = nb
        if k in write:
            v['write_bytes'] = write[k] * 1024
        if 'fetch_bytes' in v and 'write_bytes' in v:
            v['traffic'] = v['fetch_bytes'] + v['write_bytes']
            v['traffic_gbs'] = v['traffic'] / (v['avg_ms'] * 1e-3) / 1e9
    res = dict(sorted(res.items(), key=lambda kv: -kv[1]['total_ms']))
    if a.bench_json:
        line = None
        for ln in open(a.bench_json).read().splitlines():
            if ln.strip().startswith('{'):
                line = json.loads(ln)
        if line is None:
            raise SystemExit('no bench line in %s' % a.bench_json)
        res = dict({'_meta': {'lib_src': line['lib']['src'], 'workload': line['config'].get('workload_id'),
                              'mask': line['config'].get('mask'), 'continuous': line['config'].get('continuous')}},
                   **res)
    with open(a.out, 'w') as f:
        json.dump(res, f, indent=1)
    for k, v in res.items():
        if k == '_meta':
            print('# lib.src %s workload %s' % (v['lib_src'], v['workload']))
            continue
        print('%-40s n=%4d avg %.4f ms total %.3f ms%s' % (
            k[:40], v['count'], v['avg_ms'], v['total_ms'],
            ('  traffic %.3f GB' % (v['traffic'] / 1e9)) if 'traffic' in v else ''))


if __name__ == '__main__':
    main()
