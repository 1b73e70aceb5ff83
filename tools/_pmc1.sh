cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
grep -oE "(SQC?_[A-Z_0-9]+|TCP_[A-Z_0-9]+)" gpurun_out/counters_list.txt | sort -u > gpurun_out/counters_names.txt || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc1 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc1.log 2>&1
