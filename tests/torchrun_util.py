"""Launch a worker script under `torch.distributed.run` on 127.0.0.1 (the GPU data-parallel tests).

The master port is picked free and then released, so another socket can take it before the
launcher's store binds it. The launcher then fails at rendezvous with EADDRINUSE, before any
worker starts and before anything touches the GPU. Only that failure is launched again, on a
new port, at most three times. Every other failure is returned as it is.
"""
import socket
import subprocess
import sys


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _port_race(r):
    return r.returncode != 0 and "EADDRINUSE" in r.stderr and "next_rendezvous" in r.stderr


def torchrun(script, nproc, env, cwd, timeout=300):
    for _ in range(3):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
               f"--master-port={free_port()}", str(script)]
        r = subprocess.run(cmd, env=env, cwd=cwd, capture_output=True, text=True, timeout=timeout)
        if not _port_race(r):
            return r
    return r
