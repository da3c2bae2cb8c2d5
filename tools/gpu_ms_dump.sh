# The cfg3 frame's k_ekf_MS launch shapes (UVIO_HP_DUMP_MS), then the isolated microbenchmark at the most
# frequent and the largest of them.  usage: bash tools/gpu_ms_dump.sh [TAG]
set -e
O=gpurun_out/${1:-r04v}; mkdir -p $O
UVIO_HP_DUMP_MS=1 timeout -k 10 200 python -u bench.py --steps 60 --cpu-frames 0 --no-host-feed > $O/b.json 2> $O/dump.txt
grep MSDUMP $O/dump.txt | sort | uniq -c | sort -rn > $O/shapes.txt
head -20 $O/shapes.txt
A1=$(head -1 $O/shapes.txt | awk '{print $3, $5, $7, $9, $11}')
A2=$(grep MSDUMP $O/dump.txt | sort -n -k9 | tail -1 | awk '{print $3, $5, $7, $9, $11}')
echo "most frequent: $A1   largest r: $A2"
timeout -k 10 60 build/bench_small_chain 300 $A1 > $O/mb_frequent.txt
timeout -k 10 60 build/bench_small_chain 300 $A2 > $O/mb_largest.txt
cat $O/mb_frequent.txt $O/mb_largest.txt
