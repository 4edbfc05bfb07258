# Round 5: the read pipeline's carry pool (CEC_READ_CARRY) on the GPU, then an interleaved A/B of
# the c5r stream with and without it.   bash tools/r5_carry_ab.sh <tag>
set -o pipefail
T=gpurun_out/${1:-r5e}
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_readstream.py -x -v --timeout 150 --timeout-method thread > $T/pytest_readstream.log 2>&1 || { tail -40 $T/pytest_readstream.log; exit 1; }
tail -2 $T/pytest_readstream.log
for i in 1 2; do
  for c in 1 0; do
    CEC_BENCH_CARRY=$c timeout -k 10 300 python -u bench.py --config c5r --stream-gib 256 > $T/c5r_carry${c}_$i.log 2>&1 || { tail -20 $T/c5r_carry${c}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$T/c5r_carry${c}_$i.log') if l.startswith('{')][-1]); r=d['read_repair']; print('carry=$c', d['value'], r['retried_parts'], r.get('carried_chunks'), r['chunks_loaded'], r['undecodable_parts'], d['check_vs_stored'])"
  done
done
