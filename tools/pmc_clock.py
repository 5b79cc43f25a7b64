"""Effective clock per kernel from a tools/pmc_clock.sh run: GRBM_GUI_ACTIVE cycles of each
dispatch over its kernel-trace duration (median over the dispatches of each kernel)."""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    cc = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)[0]
    cyc = collections.defaultdict(dict)
    name = {}
    for r in csv.DictReader(open(cc)):
        did = int(r['Dispatch_Id'])
        cyc[did][r['Counter_Name']] = float(r['Counter_Value'])
        name[did] = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('cc::', '')
    kt = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    dur = {}
    if kt:
        for r in csv.DictReader(open(kt[0])):
            dur[int(r['Dispatch_Id'])] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-3   # us
    per = collections.defaultdict(list)
    for did, c in cyc.items():
        if did in dur and dur[did] > 50:
            per[name[did]].append((c.get('GRBM_GUI_ACTIVE', 0) / dur[did], dur[did]))
    for n, v in sorted(per.items(), key=lambda kv: -max(x[1] for x in kv[1])):
        print('%-30s n=%3d  median %.0f MHz  (duration %.3f ms)' % (n[:30], len(v), statistics.median(x[0] for x in v),
                                                                 statistics.median(x[1] for x in v) * 1e-3))


if __name__ == '__main__':
    main()
