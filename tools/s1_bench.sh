set -e
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --also= --streams 1 --steps 5 --warmup 2 2>/dev/null | python3 -c "
import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); k=d['roofline']['kernels']
print(d['value'], {n:v['avg_us'] for n,v in k.items() if 'rowC' in n or 'rowA' in n})"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --also= 2>/dev/null | grep -o '"value": [0-9.]*'
