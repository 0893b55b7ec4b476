set -o pipefail
O=gpurun_out/r01n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU -d $PWD/$O/pmc1 -o run -- python3 tools/feat_bench.py 16384 > $O/p1.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC -d $PWD/$O/pmc2 -o run -- python3 tools/feat_bench.py 16384 > $O/p2.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_MFMA_F32 SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM SQ_IFETCH -d $PWD/$O/pmc3 -o run -- python3 tools/feat_bench.py 16384 > $O/p3.log 2>&1
rc=$?; tail -2 $O/p3.log; exit $rc
