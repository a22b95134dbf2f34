# the scalar call under IE_SMALL_ZC 0 / 1 / 2, interleaved, two processes each
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_q; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for z in 0 1 2; do
    IE_SMALL_ZC=$z timeout -k 10 200 python -u tools/exp/scalar_ab.py >> $O/scalar_ab.jsonl 2>> $O/scalar_ab.err || { tail -20 $O/scalar_ab.err; exit 1; }
  done
done
cat $O/scalar_ab.jsonl
