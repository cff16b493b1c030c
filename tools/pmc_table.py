"""Per-kernel mean of every PMC counter found under an output dir of PMC passes
(p1/, p2/, ...: tools/pmc.sh, tools/gpu_r05.sh logpmc)."""
import collections, csv, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + '/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        k = k.replace('(anonymous namespace)::', '')
        if 'lvkv::' in k:
            k = k.split('lvkv::')[1].split('(')[0]
        elif k.startswith(('lvkv_', 'ck_', 'pk_')):
            k = k.split('(')[0]
        else:
            continue
        agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k in sorted(agg):
    d = {c: sum(v) / len(v) for c, v in agg[k].items()}
    n = max(len(v) for v in agg[k].values())
    print(f"{k} (n={n})")
    print("   " + "  ".join(f"{c}={x:.4g}" for c, x in sorted(d.items())))
