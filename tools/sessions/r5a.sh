# Round-5 first GPU session: the full -m gpu suite (incl. the new receptacle-cache tests), smoke(),
# the BASELINE bench line, and bench.py --gpus N self-spawn (2 ranks rehearsed on cuda:0; the
# refusal of 2 real ranks on a 1-GPU box).
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "400|r5a_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120|r5a_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "240|r5a_bench|python bench.py --gpus 1 --steps 200 --warmup 10" \
  "240|r5a_bench_spawn2|python bench.py --gpus 2 --shared-gpu --steps 100 --warmup 10" \
  "120|r5a_bench_refuse|python bench.py --gpus 2 --steps 5; rc=\$?; echo rc=\$rc; [ \$rc -eq 1 ]"
