# GPU box facts that may explain box-to-box variance (partition modes, clocks, power cap, CU count)
rocm-smi --showcomputepartition --showmemorypartition --showpower --showmaxpower --showclocks --showperflevel 2>&1 | grep -v "^$" | grep -v "=====" | head -40
python3 -c "import torch; p=torch.cuda.get_device_properties(0); print('cus', p.multi_processor_count, 'name', p.name, 'gcn', getattr(p,'gcnArchName',''), 'mem', p.total_memory)"
