for q in 2 4; do echo "FORCE_GRAPH_QUEUES=$q"; DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 100 python tools/graph_branch_probe2.py || exit 1; done
echo "BATCH 64"; DEBUG_HIP_GRAPH_BATCH_SIZE=64 timeout -k 10 100 python tools/graph_branch_probe2.py
echo "PACKET_CAPTURE=0"; DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 100 python tools/graph_branch_probe2.py
