#!/bin/bash
# kernel timeline of the unit-protocol line at N=1 (UNITS units) and of the
# single-call line: busy time (union of kernel intervals) vs the step
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-utrace}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/units -o run -- python3 $R/bench.py --no-cpu --no-900k --units-per-gpu ${UNITS:-4} --steps 3 --warmup 1 > $O/units.json 2> $O/units.err || { echo UNITS_FAILED; tail $O/units.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/single -o run -- python3 $R/bench.py --no-cpu --no-900k --steps 3 --warmup 1 > $O/single.json 2> $O/single.err || { echo SINGLE_FAILED; tail $O/single.err; exit 1; }
python3 $R/tools/timeline.py $O/units > $O/units_timeline.txt && python3 $R/tools/timeline.py $O/single > $O/single_timeline.txt && tail -25 $O/units_timeline.txt && tail -12 $O/single_timeline.txt
