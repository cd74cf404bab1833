set -u
S="bash tools/gpu_step.sh r02a"
$S 900 tests -- python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
$S 300 smoke -- python -u -c "import __graft_entry__ as g; g.smoke()"
$S 400 bench -- python -u bench.py
$S 300 band -- python -u tools/band_balance.py
$S 120 ubench -- ./tools/ubench_lds
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S 180 pmc_lds -- rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/r02a_pmc_lds -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0
cat gpurun_out/r02a_steps.log
