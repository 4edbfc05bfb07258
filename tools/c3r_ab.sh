# A/B of the device-resident read batch (bench c3r): speculative decode on/off (S), decode LDS
# reservation in KiB (L), compacted verify on/off (C); parity tests of the read path first.
#   CFGS="S L C;..." bash tools/c3r_ab.sh
set -o pipefail
# these knobs are read only by the A/B build (make -C chunky-bits_amd/csrc ab)
export CEC_LIBRARY=${CEC_LIBRARY:-tools/ab/libchunky_ec.so}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "read_batch or resilver or reconstruct or verify" > gpurun_out/pt_read.log 2>&1 || { tail -30 gpurun_out/pt_read.log; exit 1; }
IFS=';' read -ra RUNS <<< "${CFGS:-1 0 1;1 65 1;0 0 1}"
for cfg in "${RUNS[@]}"; do
  set -- $cfg
  CEC_READ_SPECULATE=$1 CEC_SPEC_LDS_KIB=$2 CEC_VERIFY_COMPACT=$3 timeout -k 10 200 python -u bench.py --config c3r --check > gpurun_out/c3r_s$1_l$2_c$3.log 2>&1 || exit 1
done
tail -2 gpurun_out/pt_read.log
for f in gpurun_out/c3r_*.log; do echo $f $(grep -o '"ms_per_step": [0-9.]*\|"check_vs_oracle": [a-z]*' $f); done
