import json,sys
b=json.load(open(sys.argv[2]))
print(sys.argv[1], ' '.join(f"{r['batches_per_go']}:{r['ms_per_go_mean']:.4f}/{r['ms_per_go_median']:.4f}" for r in b['backend']))
