#!/bin/bash
# Tile options of the 2-pass kernels at the reference's training batch (c5, batch 2: 30 planes in one grid),
# isotropic and anisotropic: line block lines (LINE_T) x column block threads (COL_THREADS).
# usage (GPU box): bash tools/small_batch_sweep.sh TAG   -> gpurun_out/TAG_sweep.jsonl
set -o pipefail
TAG=${1:-sweep}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/${TAG}_sweep.jsonl
for iso in "--iso" ""; do
    for lt in ${LTS:-0 4 2}; do
        for ct in ${CTS:-0 512 1024}; do
            echo "== $iso LINE_T=$lt COL_THREADS=$ct"
            timeout -k 10 120 python bench.py --config c5 $iso --batch 2 --steps 20 --warmup 3 \
                --opt LINE_T=$lt --opt COL_THREADS=$ct > gpurun_out/${TAG}_one.json 2>> gpurun_out/${TAG}_sweep.err || exit $?
            python - "$iso" "$lt" "$ct" gpurun_out/${TAG}_one.json >> $O <<'EOF'
import json, sys
d = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
print(json.dumps({"iso": sys.argv[1] == "--iso", "LINE_T": int(sys.argv[2]), "COL_THREADS": int(sys.argv[3]),
                  "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "kernels": {k: round(v["total_ms_per_step"], 3) for k, v in d["kernels"].items()}}))
EOF
            tail -1 $O
        done
    done
done
