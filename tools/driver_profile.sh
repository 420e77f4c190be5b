set -e
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/drv1
mkdir -p $OUT
timeout -k 10 120 python tools/driver_bench.py 200 400 $OUT/tape > $OUT/driver.json 2> $OUT/driver.err
cat $OUT/driver.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- $ROOT/opensim-moco_amd/csrc/build/mh_driver $OUT/tape/p.tape --steps 400 --x $OUT/tape/x.bin > $OUT/prof.log 2>&1
python3 $ROOT/tools/kstats.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
