"""Table of a tools/diag/backend_ab.sh run: per config, ms per go() (mean/median) and the actor phases."""
import json,sys,glob,os
d=sys.argv[1]
for i in range(len(glob.glob(f'{d}/bench_*.json'))):
    cfg=open(f'{d}/cfg_{i}.txt').read().strip()
    try: b=json.load(open(f'{d}/bench_{i}.json'))
    except Exception as e: print(i,cfg,'ERR',e); continue
    row=[]
    for r in b['backend']:
        a=r['actor_phases_ms']
        row.append(f"{r['batches_per_go']}: {r['ms_per_go_mean']:.4f}/{r['ms_per_go_median']:.4f} (prep {a['prep_ms']:.3f} dev {a['device_ms']:.3f} fill {a['fill_ms']:.3f} sync {a['stream_syncs_per_go']:.1f})")
    print(i,cfg); print('   '+'\n   '.join(row))
