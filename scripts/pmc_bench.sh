# PMC passes (one rocprofv3 run per counter group, as MI355X_MICROARCH.md
# prescribes) over a short bench.py run, for the kernels matching $1.
# Usage: gpurun -- bash scripts/pmc_bench.sh 'field_fwd|hash|field_bwd|adam|composite' tag ["fetch write"]
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RE=${1:-field_fwd}
OUT=gpurun_out/pmc_${2:-run}
mkdir -p "$OUT"
BENCH="python3 bench.py --steps 10 --warmup 2 --psnr-views 0 --no-cpu-baseline --infer-frames 0 --quality-steps 0 --no-oracle-quality --dropin-steps 0"
pass() {
    name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" -d "$OUT/$name" -o run -f csv -- $BENCH > "$OUT/$name.log" 2>&1
    python3 scripts/pmc_summary.py "$OUT/$name" 10 > "$OUT/$name.txt"
    rm -rf "$OUT/$name"
}
PASSES=${3:-fetch write tcc sq tcp lds}
want() { case " $PASSES " in *" $1 "*) return 0;; *) return 1;; esac; }
want fetch && pass fetch FETCH_SIZE
want write && pass write WRITE_SIZE
want tcc && pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
want sqw && pass sqw SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS
want sq && pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA
want tcp && pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum
want wrq && pass wrq TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum WRITE_SIZE
want enc && pass enc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
want atom && pass atom TCC_EA0_ATOMIC_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE
want lds && pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
true
