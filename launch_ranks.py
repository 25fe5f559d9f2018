"""One process per GPU for bench.py / bench_configs.py without an outside launcher.

`python bench.py --gpus N` must time N GPUs.  torchrun sets
WORLD_SIZE / RANK / LOCAL_RANK itself; a plain `python bench.py --gpus N` has none of
them, so the parent starts N children of the same script with the torchrun
environment (MASTER_ADDR 127.0.0.1, a free port) and waits for them.  The parent
makes no GPU call: it only imports the standard library, so no HIP runtime is up in
it when the children start (they are new processes, never an exec of this one).

Children's stderr goes straight through; each child's stdout is kept in a file and
handed back, so the caller decides what to print (bench.py relays rank 0's line).
If any child fails, the others are stopped (they would wait at the barrier forever)
and the parent exits with the failing child's status.
"""
import os
import socket
import subprocess
import sys
import tempfile
import time


def world_from_env():
    w = os.environ.get("WORLD_SIZE")
    return int(w) if w else None


def resolve_world(gpus):
    """The world size this process runs in: WORLD_SIZE when a launcher set it (and
    --gpus, if given, must agree), else --gpus (default 1).  SystemExit(2) on a
    mismatch: a run that silently timed fewer GPUs than asked would be a wrong line."""
    env = world_from_env()
    if env is not None and gpus is not None and env != gpus:
        sys.stderr.write(f"--gpus {gpus} but WORLD_SIZE={env}: refusing to run\n")
        raise SystemExit(2)
    if env is not None:
        return env
    return 1 if gpus is None else gpus


def needs_spawn(gpus):
    return world_from_env() is None and gpus is not None and gpus > 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_ranks(nranks, script, argv, timeout_s=None):
    """Start `nranks` children `python script argv...` as ranks 0..n-1 of one
    torch.distributed job; returns (returncode, [stdout of rank r]).  returncode is 0
    when every child exits 0, else the first failing child's status (children still
    running then are terminated)."""
    port = str(_free_port())
    outs, procs = [], []
    for r in range(nranks):
        f = tempfile.TemporaryFile(mode="w+")
        env = dict(os.environ, WORLD_SIZE=str(nranks), RANK=str(r), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(nranks), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env, stdout=f))
        outs.append(f)
    rc = 0
    t0 = time.monotonic()
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            break
        if all(c == 0 for c in codes):
            break
        if timeout_s is not None and time.monotonic() - t0 > timeout_s:
            rc = 124
            break
        time.sleep(0.05)
    if rc != 0:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    texts = []
    for f in outs:
        f.seek(0)
        texts.append(f.read())
        f.close()
    return (rc if rc >= 0 else 128 - rc), texts
