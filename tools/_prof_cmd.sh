set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc1 -o pmc1 -- python tools/stamp_profile.py tests/golden/datasets/synth_256x512.txt 100 10 512 > gpurun_out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc2 -o pmc2 -- python tools/stamp_profile.py tests/golden/datasets/synth_256x512.txt 100 10 512 > gpurun_out/pmc2.log 2>&1 || true
find gpurun_out/pmc1 gpurun_out/pmc2 -name "*.csv" | head
