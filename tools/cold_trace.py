"""HIP API calls longer than a threshold around the first cc_label_volume of a rocprofv3
--hip-trace --kernel-trace run (tools/cold_probe.py): t = 0 at the library's first kernel.

    python tools/cold_trace.py TRACE_DIR [min_ms]
"""
import csv
import glob
import os
import sys


def rows(d, pat):
    f = glob.glob(os.path.join(d, '**', pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
    api = rows(d, '*hip_api_trace.csv')
    ker = rows(d, '*kernel_trace.csv')
    ours = [k for k in ker if 'cc::' in k['Kernel_Name'] or k['Kernel_Name'].startswith('k_')]
    t0 = min(int(k['Start_Timestamp']) for k in ours)
    first = sorted(int(k['Start_Timestamp']) for k in ours)
    print('  start     duration   call')
    for a in sorted(api, key=lambda a: int(a['Start_Timestamp'])):
        s, e = int(a['Start_Timestamp']), int(a['End_Timestamp'])
        if (e - s) * 1e-6 >= thr and s > t0 - 60e6:
            print('%8.3f ms %9.3f ms  %s' % ((s - t0) * 1e-6, (e - s) * 1e-6, a['Function']))
    print('first kernels:')
    for k in sorted(ours, key=lambda k: int(k['Start_Timestamp']))[:24]:
        s, e = int(k['Start_Timestamp']), int(k['End_Timestamp'])
        print('%8.3f ms %9.3f ms  %s' % ((s - t0) * 1e-6, (e - s) * 1e-6, k['Kernel_Name'][:60]))


if __name__ == '__main__':
    main()
