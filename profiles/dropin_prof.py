"""The drop-in latency loop alone (bench.frame_latency: qpsk_rx_frame() call by
call), for a kernel trace of the per-frame path:
    rocprofv3 --kernel-trace --stats -d gpurun_out/dropin -- python3 profiles/dropin_prof.py 512"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(json.dumps(bench.frame_latency(int(sys.argv[1]) if len(sys.argv) > 1 else 512, 1)))
