set -e
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/pmc
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv -d $R/gpurun_out/pmc/a -o run -- python3 bench.py --config table --compression 1 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/a.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/pmc/b -o run -- python3 bench.py --config table --compression 1 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/b.log 2>&1
find gpurun_out/pmc -name "*counter_collection.csv" | head
