# Counter passes over the fused encode+CRC (default + factored variant) and
# the encode kernel: clock (GRBM_GUI_ACTIVE vs duration), instruction mix,
# LDS bank conflicts. One --pmc pass per run (rocprofv3 does not split).
set -o pipefail
O=$(pwd)/gpurun_out/pmcf
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
cd /tmp
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
for v in 2 3; do
  HRS_FUSED=$v timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES \
    -d $O/a_v$v -o run -- python3 $R/tools/bench_encode_crc.py --iters 5 > $O/a_v$v.log 2>&1 || exit $?
  HRS_FUSED=$v timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY \
    -d $O/b_v$v -o run -- python3 $R/tools/bench_encode_crc.py --iters 5 > $O/b_v$v.log 2>&1 || exit $?
done
