# Same-box timing of ab/*.so without the GPU suite (timing probes whose results are not meant to be exact).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
REPS=${REPS:-3} bash scripts/ab_run.sh ${1:-abt} ${2:-2} > /dev/null || exit 1
python scripts/ab_table.py gpurun_out/${1:-abt}/ab.log
