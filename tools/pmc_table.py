"""Print per-kernel SQ counters from a tools/pmc_ablate.sh run (first dispatch of each kernel),
normalised per tile (131072 tiles at C3 unless --tiles)."""
import collections, csv, glob, sys
d = sys.argv[1]
tiles = float(sys.argv[2]) if len(sys.argv) > 2 else 131072
f = glob.glob(d + '/**/*counter_collection.csv', recursive=True)[0]
per = collections.OrderedDict()
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('cc::', '')
    key = (int(r['Dispatch_Id']), n)
    per.setdefault(key, {})[r['Counter_Name']] = float(r['Counter_Value'])
seen = set()
cols = ['SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_LDS_BANK_CONFLICT', 'SQ_WAIT_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAVE_CYCLES', 'SQ_INSTS_VMEM_RD']
print('%-34s' % 'kernel (per tile)' + ''.join('%12s' % c.replace('SQ_', '')[:11] for c in cols))
for (did, n), v in sorted(per.items()):
    if n in seen or n.startswith('__amd') or 'generate' in n:
        continue
    seen.add(n)
    print('%-34s' % n[:34] + ''.join('%12.0f' % (v.get(c, 0) / tiles) for c in cols))
