import csv, glob, sys
for v in sys.argv[1:]:
    f = glob.glob(f"gpurun_out/itxs_{v}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted((r for r in csv.DictReader(open(f)) if 'itx_frame_kernel' in r['Kernel_Name']), key=lambda r: int(r['Start_Timestamp']))
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows]
    out, i = [], 0
    for nm in ['all'] + [f'tx{s}' for s in range(19)]:
        c = sorted(d[i:i + 53]); i += 53
        if c: out.append(f"{nm}:{c[len(c) // 2]:.1f}")
    print(v, ' '.join(out))
