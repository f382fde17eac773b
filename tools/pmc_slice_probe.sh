set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/spp
for c in "TCC_HIT TCC_MISS" "TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD" ; do
  n=$(echo $c | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $c -T -d gpurun_out/spp/$n -o run --output-format csv -- python3 tools/slice_probe.py --steps 3 > gpurun_out/spp/$n.log 2>&1 || echo "fail $c"
done
echo done
