set -o pipefail
O=gpurun_out/fused5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 1 2; do
  HRS_FUSED=$v timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_v$v -o run -- python tools/bench_encode_crc.py --iters 2 > $O/pmc_v$v.txt 2>&1 || exit $?
done
