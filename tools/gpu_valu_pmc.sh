# VALU / wait counters per kernel over a short default bench (one --pmc pass)
set -e
O=gpurun_out/${1:-valu_pmc}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --timer-every 1000000 > $R/$O/pmc.log 2>&1
