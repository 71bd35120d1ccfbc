"""Launch a worker script under `torch.distributed.run` on 127.0.0.1 (the GPU data-parallel tests).

The launcher picks its own port: `--standalone` runs a c10d rendezvous whose store binds port 0
on 127.0.0.1 (`--local-addr`), so the port is taken by the socket that uses it and no other
process can claim it in between (the round-5 helper picked a free port, released it and handed
the number on, a check-then-use race it then had to retry).  The workers reach the launcher's
store through the MASTER_ADDR / MASTER_PORT it exports to them.
"""
import subprocess
import sys


def torchrun_cmd(script, nproc):
    return [sys.executable, "-m", "torch.distributed.run", "--standalone",
            "--local-addr=127.0.0.1", f"--nproc-per-node={nproc}", str(script)]


def torchrun(script, nproc, env, cwd, timeout=300):
    return subprocess.run(torchrun_cmd(script, nproc), env=env, cwd=cwd, capture_output=True,
                          text=True, timeout=timeout)
