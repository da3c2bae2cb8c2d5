# rocprofv3 kernel statistics of one bench workload for the current library and another build (UVIO_HP_LIB).
# usage: bash tools/gpu_kstats_ab.sh OTHER_LIB OUTDIR workload
set -e
R=$GRAFT_REPO_ROOT
B=$1; O=$R/gpurun_out/$2; WL=$3
cd $R && mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o run -- python3 $R/bench.py --workload $WL --steps 200 --cpu-frames 0 > $O/new.json 2> $O/new.err)
(cd /tmp && UVIO_HP_AB_OLD=1 UVIO_HP_LIB=$R/$B timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/old -o run -- python3 $R/bench.py --workload $WL --steps 200 --cpu-frames 0 > $O/old.json 2> $O/old.err)
python tools/prof_summary.py $O/new/run_kernel_trace.csv > $O/new_per_frame.txt
python tools/prof_summary.py $O/old/run_kernel_trace.csv > $O/old_per_frame.txt
rm -f $O/new/run_kernel_trace.csv $O/old/run_kernel_trace.csv
