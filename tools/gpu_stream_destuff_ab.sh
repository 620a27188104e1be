set -e
cd $GRAFT_REPO_ROOT
for pin in 1 0 1 0; do
  HJD_STREAM_PINNED=$pin timeout -k 10 300 python bench.py --workload stream4k420 --steps 3 --warmup 1 > gpurun_out/stream_pin$pin.json 2> gpurun_out/stream_pin$pin.err
  python3 -c "import json; d=json.load(open('gpurun_out/stream_pin$pin.json')); print('pinned=$pin', d['value'], d['end_to_end'])"
done
