set -x
nproc; cat /sys/fs/cgroup/cpu.max; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; lscpu | head -30
rocm-smi --showbus 2>/dev/null | head -20
python3 -c "
import torch
p=torch.cuda.get_device_properties(0); print(p); print([a for a in dir(p) if 'pci' in a])
print(p.pci_bus_id, p.pci_device_id, p.pci_domain_id)
"
ls /sys/bus/pci/devices | head -50
for d in /sys/bus/pci/devices/*; do if [ -f $d/numa_node ] && grep -q 0x1002 $d/vendor 2>/dev/null; then echo $d $(cat $d/class) $(cat $d/numa_node) $(cat $d/local_cpulist); fi; done
numactl -H 2>/dev/null | head
cat /sys/devices/system/node/node*/cpulist
