#!/bin/bash
# Round 4: (1) the G20 link gap -- launch-mode zero-copy kernels, throughput and two rocprofv3
# counter passes per case; (2) config 5 on the durable broker: 60 s JSON at
# 1.2e6 tx/s without and with a kafka-lite SIGKILL + restart from disk at t = 25 s (next #4).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O/g20
step() { echo "[r4e] $(date +%T) $*"; }
df -h /tmp . > $O/df.txt 2>&1; cat $O/df.txt
step kernel_sol host zero-copy
timeout -k 10 240 python bench/kernel_sol.py --host --cases gbdt:g20,gbdt:g32,mlp:w64 --sizes 65536,1048576,16777216 \
  --iters 10 --out $O/g20/kernel_sol_host.json > $O/g20/kernel_sol_host.log 2>&1 || { tail -30 $O/g20/kernel_sol_host.log; exit 1; }
grep '"rows": 16777216' $O/g20/kernel_sol_host.log
PA="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_IO_CREDIT_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_64B_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
PB="TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum TCC_UC_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_UC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
for case in gbdt:g20 mlp:w64; do
  tag=${case/:/_}
  for pass in A B; do
    [ $pass = A ] && P="$PA" || P="$PB"
    step pmc $case pass $pass
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/g20/pmc_${tag}_$pass -o run -- \
      python3 bench/kernel_sol.py --host --cases $case --sizes 16777216 --iters 3 > $O/g20/pmc_${tag}_$pass.log 2>&1 \
      || { tail -20 $O/g20/pmc_${tag}_$pass.log; exit 1; }
  done
done
find $O/g20 -name '*counter_collection.csv' | head
step json 60 s durable, no kill
timeout -k 30 420 python bench/deploy_topology.py --seconds 60 --producers 3 --rate 1200000 --fmt json \
  --log-dir $O/json60 --out $O/topo_json60_durable.json > $O/topo_json60_durable.log 2>&1 \
  || { tail -40 $O/topo_json60_durable.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/topo_json60_durable.json')); print(d['value'], d['min_sample_tx_s'], d['checks_passed'], d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], d.get('produce_to_scored_us'), d.get('scored_to_process_started_us'), d.get('kafka_data_bytes'))"
step json 60 s, kafka-lite SIGKILLed at 25 s
timeout -k 30 480 python bench/deploy_topology.py --seconds 60 --producers 3 --rate 1200000 --fmt json \
  --kafka-kill-at 25 --kafka-down-s 2 --log-dir $O/json60_kill --out $O/topo_json60_kafka_kill.json \
  > $O/topo_json60_kafka_kill.log 2>&1 || { tail -40 $O/topo_json60_kafka_kill.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/topo_json60_kafka_kill.json')); print(d['value'], d['checks_passed'], d['incoming_equals_produced'], d['kie_duplicates'], d.get('kafka_outage'), [s['tx_s'] for s in d['samples']])"
step done
