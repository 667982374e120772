#!/bin/bash
# Round 4: is the durable broker's JSON fetch p99 (~20 ms vs ~6 ms in memory) the box's disk
# writeback?  The same JSON run with kafka-lite's data directory on the box's disk ($TMPDIR =
# /tmp) and on tmpfs (/dev/shm: page cache without writeback), when /dev/shm has the room.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4t
mkdir -p $O
step() { echo "[r4t] $(date +%T) $*"; }
df -h /tmp /dev/shm | tee $O/df.txt
free_gb=$(df --output=avail -BG /dev/shm | tail -1 | tr -dc '0-9')
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['min_sample_tx_s'], 'checks', d['checks_passed'], 'durable', d.get('kafka_durable'), 'bytes', d.get('kafka_data_bytes'))
print('produce->scored', d['produce_to_scored_us'])" "$1"; }
step json, data on disk
TMPDIR=/tmp timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 3 --rate 1200000 --fmt json \
  --retention-batches 100 --log-dir $O/disk --out $O/json_disk.json > $O/json_disk.log 2>&1 || { tail -40 $O/json_disk.log; exit 1; }
show $O/json_disk.json
if [ "${free_gb:-0}" -ge 16 ]; then
  step json, data on tmpfs
  TMPDIR=/dev/shm timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 3 --rate 1200000 --fmt json \
    --retention-batches 100 --log-dir $O/shm --out $O/json_shm.json > $O/json_shm.log 2>&1 || { tail -40 $O/json_shm.log; exit 1; }
  show $O/json_shm.json
else
  echo "[r4t] /dev/shm has ${free_gb} GB free: tmpfs run skipped"
fi
step done
