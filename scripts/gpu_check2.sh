# 2-rank shared-GPU rehearsals of the sharded bench at B and C (pair-split selection, range ingest)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/shard_rehearsal.sh B || { echo "rehearsal B rc=$?"; tail -20 gpurun_out/shard2_B.log; exit 1; }
bash scripts/shard_rehearsal.sh C || { echo "rehearsal C rc=$?"; tail -20 gpurun_out/shard2_C.log; exit 1; }
echo ALLDONE
