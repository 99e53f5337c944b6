# r04aa: the pipelined calls' second stream at normal and at the highest priority, in a process
# with and without a one-rank RCCL group (its streams compete for the hardware queues)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/prio_0.so ab/prio_1.so --rounds 5 --legs symbols2image,zerorun_encode > gpurun_out/r04aa_ab_plain.log 2>&1 || { tail -20 gpurun_out/r04aa_ab_plain.log; exit 1; }
tail -6 gpurun_out/r04aa_ab_plain.log
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/prio_0.so ab/prio_1.so --rounds 5 --legs symbols2image,zerorun_encode --rccl > gpurun_out/r04aa_ab_rccl.log 2>&1 || { tail -20 gpurun_out/r04aa_ab_rccl.log; exit 1; }
tail -6 gpurun_out/r04aa_ab_rccl.log
