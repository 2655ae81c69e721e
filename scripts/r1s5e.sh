#!/bin/bash
# polled vs blocking host syncs: GPU suite, then the bench both ways
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r1s5e_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r1s5e_pytest.log; exit 1; }
tail -2 gpurun_out/r1s5e_pytest.log
for v in poll block; do
    e=""; [ $v = block ] && e="block"
    SLAMHIP_SYNC=$e timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r1s5e_$v.json 2> gpurun_out/r1s5e_$v.err || exit 2
done
python - <<'PY'
import json
for t in ("poll", "block"):
    for line in open(f"gpurun_out/r1s5e_{t}.json"):
        if line.startswith("{"):
            d = json.loads(line)
    print(t, round(d["value"], 1), round(d["ms_per_step"], 3), "orb", round(d["orb"]["frames_per_s"]), "ba8", round(d["ba_window"]["ms_per_window"], 2),
          "ba16", round(d["ba_window_w16_4k"]["ms_per_window"], 2), "pipe", round(d["pipeline"]["frames_per_s"], 1), d["pipeline"]["ms_by_op"],
          "4k", round(d["sift_4k"]["frames_per_s"]), "det", round(d["sift_detector"]["ms_per_frame"], 2))
PY
