"""Print bench.kernel_src_sha256(): the hash of k_relax's sources and hipcc flags that a PMC
profile directory records in src.sha256 (tools/gpu_r03c.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(bench.kernel_src_sha256())
