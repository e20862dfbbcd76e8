cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5s34; mkdir -p $O
B="--gpus 1 --steps 20 --warmup 5 --cpu-baseline off --critical-path off --reference-loop off --single-frame off"
for r in 1 2 3 4; do
for cfg in "0 0" "10 2" "10 3" "12 2" "14 2" "16 1"; do
set -- $cfg
timeout -k 10 120 python bench.py $B --batch $1 --inflight $2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
grep '^{' $O/b.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$r', '$1x$2', d['value'], d['ms_per_step'], d['config'].get('launch_sizes'))" | tee -a $O/shape.txt
done; done
echo done
