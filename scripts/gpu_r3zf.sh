set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3zf; mkdir -p $O; R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $R/$O/p1 -o p1 -- python3 $R/bench/gibbs_ab.py --topics 20 --burn 150 --rounds 1 --sweeps 3 --modes wdelta+q2 > $R/$O/p1.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d $R/$O/p2 -o p2 -- python3 $R/bench/gibbs_ab.py --topics 20 --burn 150 --rounds 1 --sweeps 3 --modes wdelta+q2 > $R/$O/p2.log 2>&1
