set -o pipefail
export TMPDIR=/tmp
bash tools/pmc_libs.sh gpurun_out/r7d/p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" ab/lib_base.so slam_framework_amd/libslamgpu.so && \
bash tools/pmc_libs.sh gpurun_out/r7d/p2 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE" ab/lib_base.so slam_framework_amd/libslamgpu.so
