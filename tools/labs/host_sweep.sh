# Host-buffer call rates vs chunk size and copy threads (each config its own process).
mkdir -p gpurun_out/host
for t in 0 2 4 8; do
  for ch in 262144 524288 1048576; do
    HRS_HOST_THREADS=$t HRS_HOST_CHUNK=$ch timeout -k 10 120 python tools/bench_host_api.py --calls 30 > gpurun_out/host/t${t}_c${ch}.json 2>&1 || exit $?
  done
done
