cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04k
timeout -k 10 200 python -u bench.py --stamps --steps 400 --warmup 20 > gpurun_out/r04k/stamps_head.json 2>&1 || exit $?
KB_STAMPS_LIB=$PWD/kafkabalancer_amd/lib/libkbengine_stampsfrz.so timeout -k 10 200 python -u bench.py --stamps --steps 400 --warmup 20 > gpurun_out/r04k/stamps_frz.json 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --stamps --steps 400 --warmup 20 > gpurun_out/r04k/stamps_head2.json 2>&1 || exit $?
python3 - <<'PY'
import json
rows = {}
for n in ("frz", "head", "head2"):
    d = [json.loads(l) for l in open("gpurun_out/r04k/stamps_%s.json" % n) if l.startswith("{")][0]
    rows[n] = d
ks = list(rows["head"]["stamps_us_per_step"])
print("%-18s %8s %8s %8s" % ("phase", "frz", "head", "head2"))
for k in ks:
    print("%-18s %8.3f %8.3f %8.3f" % (k, rows["frz"]["stamps_us_per_step"].get(k, 0), rows["head"]["stamps_us_per_step"][k], rows["head2"]["stamps_us_per_step"][k]))
print("k_step_us", rows["frz"]["k_step_us"], rows["head"]["k_step_us"], rows["head2"]["k_step_us"])
PY
