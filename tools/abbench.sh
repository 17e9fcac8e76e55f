set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for l in base nto; do
  ACX_LIB=$PWD/abx/lib_$l.so timeout -k 10 120 python -u bench.py --no-cpu --no-step-api > gpurun_out/abb_${l}_${i}.log 2>&1 || exit 1
  echo $l $i $(tail -1 gpurun_out/abb_${l}_${i}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'])")
done
done
