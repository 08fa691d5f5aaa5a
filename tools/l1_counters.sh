set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1; echo "list rc=$?"
grep -o "^[A-Za-z_0-9]*\|[ \t]TCP_[A-Z_0-9]*\|TA_[A-Z_0-9]*\|TD_[A-Z_0-9]*\|TCC_[A-Z_0-9]*" gpurun_out/avail.txt | sort -u | head -0
bash tools/pmc_kernel.sh gpurun_out/l1c "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
