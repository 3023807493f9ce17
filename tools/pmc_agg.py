import csv, sys, collections, glob
tag = sys.argv[1]; kern = sys.argv[2] if len(sys.argv) > 2 else 'pathtrace_kernel<false'
for p in sorted(glob.glob(f"gpurun_out/{tag}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(p)):
        if kern in r['Kernel_Name']:
            agg[r['Counter_Name']] += float(r['Counter_Value'])
    print(p.split('/')[2], {k: f"{v:.4g}" for k, v in sorted(agg.items())})
