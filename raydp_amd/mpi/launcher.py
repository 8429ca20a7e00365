"""Built-in MPI process launcher, used when no ``mpirun`` is installed.

It understands the subset of ``mpirun`` flags the job classes emit (``-hosts``/``-H``,
``-ppn``/``-N``/``-n``/``-np``, ``-prepend-rank``/``--tag-output``, ``-genv K V``/``-x K``)
and starts every rank on this machine with the rank variables the chosen MPI flavour exports
(reference consumers: ``python/raydp/mpi/mpi_worker.py`` get_rank — OMPI_COMM_WORLD_RANK /
_LOCAL_RANK for Open MPI, PMI_RANK / MPI_LOCALRANKID for Intel MPI and MPICH). Output is
forwarded with a ``[rank]`` prefix. Any rank failing terminates the others and the launcher
exits with that rank's code, which is what ``mpirun`` does.

Usage: ``python -m raydp_amd.mpi.launcher --mpi-type mpich -hosts a,b -ppn 2 -- prog args``
"""
import argparse
import os
import signal
import subprocess
import sys
import threading
from typing import Dict, List, Optional, Tuple

FLAVOURS = {
    "openmpi": ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "OMPI_COMM_WORLD_SIZE",
                "OMPI_COMM_WORLD_LOCAL_SIZE"),
    "intel_mpi": ("PMI_RANK", "MPI_LOCALRANKID", "PMI_SIZE", "MPI_LOCALNRANKS"),
    "mpich": ("PMI_RANK", "MPI_LOCALRANKID", "PMI_SIZE", "MPI_LOCALNRANKS"),
}


def parse_mpirun(argv: List[str]) -> Tuple[List[str], int, Optional[int], bool, Dict[str, str], List[str]]:
    """(hosts, ppn, np, prefix, env, program) from an ``mpirun`` command line (without argv[0])."""
    hosts: List[str] = []
    ppn, np_, prefix, env = 1, None, False, {}
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ("-hosts", "-H", "--host", "-host"):
            hosts = [h.split(":")[0] for h in argv[i + 1].split(",") if h]
            i += 2
        elif a in ("-ppn", "-N", "--npernode", "-npernode"):
            ppn = int(argv[i + 1])
            i += 2
        elif a in ("-n", "-np", "--np"):
            np_ = int(argv[i + 1])
            i += 2
        elif a in ("-prepend-rank", "--tag-output", "-l"):
            prefix = True
            i += 1
        elif a in ("-genv", "-env"):
            env[argv[i + 1]] = argv[i + 2]
            i += 3
        elif a == "-x":
            k, _, v = argv[i + 1].partition("=")
            if v or k not in os.environ:
                env[k] = v
            else:
                env[k] = os.environ[k]
            i += 2
        elif a == "--":
            return hosts, ppn, np_, prefix, env, argv[i + 1:]
        elif a.startswith("-"):
            i += 1  # flags without values we do not model (e.g. --allow-run-as-root)
        else:
            return hosts, ppn, np_, prefix, env, argv[i:]
    return hosts, ppn, np_, prefix, env, []


def launch(program: List[str], hosts: List[str], ppn: int, mpi_type: str, prefix: bool = True,
           env: Optional[Dict[str, str]] = None, np_: Optional[int] = None) -> int:
    from raydp_amd.mpi.utils import local_addresses
    hosts = hosts or ["127.0.0.1"]
    mine = set(local_addresses()) | {"localhost", os.uname().nodename}
    remote = [h for h in hosts if h not in mine]
    if remote:
        raise RuntimeError(f"built-in launcher runs ranks on this machine only; remote hosts {remote} "
                           "need a real mpirun")
    world = np_ if np_ is not None else ppn * len(hosts)
    rk, lrk, sz, lsz = FLAVOURS[mpi_type]
    procs: List[subprocess.Popen] = []
    lock = threading.Lock()
    for r in range(world):
        e = dict(os.environ)
        e.update(env or {})
        e.update({rk: str(r), lrk: str(r % ppn), sz: str(world), lsz: str(ppn)})
        procs.append(subprocess.Popen(program, env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))

    def pump(r, p):
        for line in iter(p.stdout.readline, b""):
            with lock:
                sys.stdout.write((f"[{r}] " if prefix else "") + line.decode(errors="replace"))
                sys.stdout.flush()

    threads = [threading.Thread(target=pump, args=(r, p), daemon=True) for r, p in enumerate(procs)]
    for t in threads:
        t.start()

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
        sys.exit(128 + sig)

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            try:
                code = p.wait(timeout=0.05)
            except subprocess.TimeoutExpired:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # one rank failed: abort the job like mpirun does
                    q.terminate()
    for t in threads:
        t.join(1)
    return rc


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--mpi-type", default="mpich", choices=sorted(FLAVOURS))
    known, rest = ap.parse_known_args(argv)
    hosts, ppn, np_, prefix, env, program = parse_mpirun(rest)
    if not program:
        print("usage: launcher --mpi-type T [mpirun flags] -- program args", file=sys.stderr)
        return 2
    return launch(program, hosts, ppn, known.mpi_type, prefix, env, np_)


if __name__ == "__main__":
    sys.exit(main())
