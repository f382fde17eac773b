set -e
for sub in 16384 32768 65536; do
  LGCN_RECALL_SUBSET=$sub timeout -k 10 200 python tools/eval_probe.py --reps 3 > gpurun_out/ev_$sub.log 2>&1
  LGCN_RECALL_SUBSET=$sub timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d gpurun_out/evp_$sub -o run --output-format csv -- python3 tools/eval_probe.py --reps 2 > /dev/null 2>&1
done
echo done
