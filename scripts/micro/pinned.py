"""Run a command as a child process on the CPUs of GPU 0's NUMA node (the
bench's pinning, bench.py pin_host):  python scripts/micro/pinned.py CMD ..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402

print("#", bench.pin_host(0), flush=True)
sys.exit(subprocess.call(sys.argv[1:]))
