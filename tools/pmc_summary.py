"""Summarise rocprofv3 --pmc CSVs per kernel variant (mean over dispatches)."""
import collections, csv, glob, sys
base = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(base + '/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if 'crc32c_batch' in k:
            name = 'crc_v' + (k.split('<')[1].split('>')[0] if '<' in k else '?')
        elif 'read_bw_dword' in k:
            name = 'readbw_dword'
        elif 'read_bw' in k:
            name = 'readbw16'
        else:
            continue
        agg[name][r['Counter_Name']].append(float(r['Counter_Value']))
for name in sorted(agg):
    d = {c: sum(v) / len(v) for c, v in agg[name].items()}
    print(name, ' '.join(f"{c}={x:.4g}" for c, x in sorted(d.items())))
