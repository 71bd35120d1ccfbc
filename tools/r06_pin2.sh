#!/bin/bash
# Round 6 (gpurun_out/r06q/): where the staging threads run (IMPALA_STAGE_PIN): the GPU's NUMA
# node (default), the caller's node, anywhere; three processes each, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
Q="--steps 20 --warmup 5 --no-alt-line --no-cpu-baseline"
python3 -c "
import torch, os
p = torch.cuda.get_device_properties(0)
bus = '%04x:%02x:%02x.0' % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
print('gpu', bus, open('/sys/bus/pci/devices/%s/numa_node' % bus).read().strip())"
for i in 1 2 3; do
for v in gpu caller 0; do
  IMPALA_STAGE_PIN=$v timeout -k 10 300 python bench.py $Q > $O/$v$i.json 2> $O/$v$i.err; rc=$?; fatal $rc $v$i
  python3 -c "import json;d=json.load(open('$O/$v$i.json'));l=d['learner_loop']['host_list_replay'];print('$v run $i', 'hs', d['host_staged']['ms_per_step'], 'list', {k:(v['ms_per_step'],v['ms_per_step_median'],v['host_ms_per_iter_median']) for k,v in l.items()})"
done
done
