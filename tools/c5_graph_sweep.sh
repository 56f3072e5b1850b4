set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
O=gpurun_out/r05h_c5.jsonl
for a in "--iso --batch 2" "--iso --batch 2 --graph" "--iso --batch 2 --graph --no-merge" "--batch 2" "--batch 2 --graph" "--batch 2 --graph --no-merge" "--iso --batch 64 --graph" "--batch 64 --graph"; do
  echo "== $a" | tee -a gpurun_out/r05h_c5.log
  timeout -k 10 240 python bench.py --config c5 $a --steps 10 --warmup 3 >> $O 2>> gpurun_out/r05h_c5.log || { echo "rc=$? for $a"; exit 1; }
  tail -1 $O | cut -c1-200
done
