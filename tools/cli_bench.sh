# rgbd_mmt end to end on a synthetic sequence in the reference's layout: decode (PNG, .flo, text
# masks) on host threads + chunked tracking, against frame-by-frame with one decode thread.
# Usage: cli_bench.sh [frames]
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${1:-400}
SEQ=/tmp/mmt_cli_seq
timeout -k 10 400 python tools/make_synth_sequence.py $SEQ $N --device cuda > gpurun_out/cli_gen.log 2>&1
EXE=multimot_track_amd/rgbd_mmt
for cfg in "--chunk 1 --threads 1" "--chunk 1 --threads 16" "--chunk 16 --threads 16" "--chunk 32 --threads 16"; do
  timeout -k 10 300 $EXE ORBvoc.txt $SEQ/settings.yaml $SEQ $cfg > gpurun_out/cli_run.txt 2> gpurun_out/cli_run.err
  echo "$cfg: $(grep -E 'end-to-end|mean tracking' gpurun_out/cli_run.txt | tr '\n' ' ')"
done
rm -rf $SEQ
