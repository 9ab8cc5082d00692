"""The C examples built with plain gcc against include/ + libpptkrx.so and run
over the golden sets (examples/rxq_file.h frame-set files written here):

  examples/rx_mt.c        one thread + one pptk_rx_ctx per rx queue
                          (reference ldp/ldprecvmt.c:16-67), pptk_rx_batch;
  examples/rx_multigpu.c  one thread per GPU, one RCCL communicator over all
                          of them (pptk_rx_comm_create_all), sharded device
                          batches and the in-place flow-hash all-gather;
  examples/rx_perf.c      device-resident throughput from C (ipcksumperf's
                          GPU counterpart), checked against the host APIs.

Both compare every record (and the gathered hash array) with the
reference-made golden records, so a passing run is bit-exact parity."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_golden

INCLUDE = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "pptk_amd")
SETS = ("edge", "fuzz", "cmix", "c64")


def write_rxq(path, names=SETS):
    """Concatenate golden sets into one frame-set file (rxq_file.h)."""
    bufs, offs, lens, recs, pos = [], [], [], [], 0
    key = None
    for name in names:
        z = load_golden(name)
        key = z["key"].tobytes()
        bufs.append(z["buf"])
        offs.append(z["off"].astype(np.uint64) + np.uint64(pos))
        lens.append(z["len"].astype(np.uint16))
        recs.append(z["recs"])
        pos += len(z["buf"])
    off, ln = np.concatenate(offs), np.concatenate(lens)
    buf = np.concatenate(bufs)
    hdr = np.zeros(1, dtype=[("magic", "<u4"), ("n", "<u4"), ("buf_bytes", "<u8"),
                             ("key", "u1", 16)])
    hdr["magic"], hdr["n"], hdr["buf_bytes"] = 0x31515852, len(off), len(buf)
    hdr["key"] = np.frombuffer(key, np.uint8)
    with open(path, "wb") as f:
        for a in (hdr, off, ln, buf, np.concatenate(recs)):
            f.write(a.tobytes())
    return len(off)


def build(tmp_path, name, hip=False):
    exe = str(tmp_path / name)
    cmd = ["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-Werror", "-pthread", "-I", INCLUDE]
    if hip:
        cmd += ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
    cmd += [os.path.join(ROOT, "examples", f"{name}.c"), "-L", LIBDIR, "-lpptkrx",
            f"-Wl,-rpath,{LIBDIR}"]
    if hip:
        cmd += ["-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.check_call(cmd + ["-o", exe])
    return exe


def test_examples_build(tmp_path):
    build(tmp_path, "rx_mt")
    build(tmp_path, "rx_multigpu", hip=True)
    build(tmp_path, "rx_perf", hip=True)
    build(tmp_path, "rx_loop")


def test_rxq_file_layout(tmp_path):
    p = str(tmp_path / "s.rxq")
    n = write_rxq(p, ("edge",))
    z = load_golden("edge")
    raw = open(p, "rb").read()
    assert len(raw) == 32 + n * (8 + 2 + 64) + len(z["buf"])
    assert np.frombuffer(raw[:4], "<u4")[0] == 0x31515852


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["", "pipe", "rec32", "pipe32"])
@pytest.mark.parametrize("threads", [1, 4, 8])
def test_rx_mt_threads_bit_exact(tmp_path, threads, mode):
    """N rx threads, each with its own context and queue, 2 laps, bursts
    synchronous or two in flight per thread, 64- or 32-byte records
    (pptk_rx_batch32 / _submit32 from a C host): every record equals the
    golden record (or its compact form)."""
    p = str(tmp_path / "s.rxq")
    n = write_rxq(p)
    out = subprocess.run([build(tmp_path, "rx_mt"), p, str(threads), "2"] + ([mode] if mode else []),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    tag = (" (pipelined)" if mode.startswith("pipe") else "") + \
        (" (32-byte records)" if mode.endswith("32") else "")
    assert f"{threads} threads{tag}, {2 * n} frames" in out.stdout and "0 mismatches" in out.stdout


@pytest.mark.gpu
def test_rx_multigpu_allgather_bit_exact(tmp_path):
    """One thread per visible GPU, one communicator over them: every GPU's
    records and the whole gathered hash array equal the golden records."""
    p = str(tmp_path / "s.rxq")
    n = write_rxq(p)
    out = subprocess.run([build(tmp_path, "rx_multigpu", hip=True), p], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert f"{n} frames, 0 mismatches" in out.stdout


@pytest.mark.gpu
def test_rx_multigpu_split_overlap_bit_exact(tmp_path):
    """split_cus 32 (4th argument; no environment knob, no RCCL variable):
    the gathers on their own stream beside the next batch, the chip's CUs
    split between the two (pptk_rx_stream_split, made before the
    communicator, which the library then caps at 32 channels), batch r
    waiting for gather r - 2; four rounds, bit-exact as above.  The streams
    are the context's: the example's pptk_rx_stream_destroy of the gather
    stream before pptk_rx_ctx_destroy -- the order that hung in round 5 --
    returns EBUSY, and the context's own teardown (communicator first, then
    its streams) ends the process cleanly."""
    p = str(tmp_path / "s.rxq")
    n = write_rxq(p)
    env = dict(os.environ, RX_MULTIGPU_TRACE="1", RX_MULTIGPU_TIMEOUT_MS="20000")
    env.pop("NCCL_MAX_NCHANNELS", None)
    exe = build(tmp_path, "rx_multigpu", hip=True)
    with open(tmp_path / "out", "w+") as fo, open(tmp_path / "err", "w+") as fe:
        pr = subprocess.Popen([exe, p, "1", "4", "32"], stdout=fo, stderr=fe, env=env)
        try:
            rc = pr.wait(timeout=90)
        except subprocess.TimeoutExpired:
            pr.kill()
            pr.wait()
            rc = "killed"
        fo.seek(0)
        fe.seek(0)
        out, err = fo.read(), fe.read()
    assert rc == 0, (rc, out, err)
    assert f"{n} frames, 0 mismatches" in out
    assert "before the context: -16 (EBUSY" in out, out


@pytest.mark.gpu
def test_rx_multigpu_thread_join_bit_exact(tmp_path):
    """The per-process join form in threads (RX_MULTIGPU_JOIN=threads: a uid
    from main, pptk_rx_comm_create in every rank's thread), one rank per GPU:
    bit-exact as above."""
    p = str(tmp_path / "s.rxq")
    n = write_rxq(p)
    env = dict(os.environ, RX_MULTIGPU_JOIN="threads")
    out = subprocess.run([build(tmp_path, "rx_multigpu", hip=True), p], capture_output=True,
                         text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    assert f"{n} frames, 0 mismatches" in out.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("join,ranks", [("all", 1), ("threads", 2)])
def test_rx_multigpu_failed_thread_exits_nonzero(tmp_path, join, ranks):
    """Failure containment: the last rank's thread fails (RX_MULTIGPU_FAIL).
    create_all form: it fails before its first gather and aborts every
    communicator.  Thread-join form, two ranks: it fails instead of joining
    and aborts every context, so rank 0's pptk_rx_comm_create -- whether
    already waiting or not yet called -- returns ECANCELED (-125) at once
    instead of waiting for the 3 s deadline.  Either way the process exits 1,
    promptly."""
    import time
    p = str(tmp_path / "s.rxq")
    write_rxq(p, ("edge",))
    env = dict(os.environ, RX_MULTIGPU_JOIN=join, RX_MULTIGPU_FAIL=str(ranks - 1),
               RX_MULTIGPU_TIMEOUT_MS="3000")
    t0 = time.monotonic()
    out = subprocess.run([build(tmp_path, "rx_multigpu", hip=True), p, str(ranks), "2"],
                         capture_output=True, text=True, timeout=120, env=env)
    took = time.monotonic() - t0
    assert out.returncode == 1, out.stdout + out.stderr
    assert "FAILED" in out.stdout and took < 60, (took, out.stdout)
    if join == "threads":
        assert "rc -125" in out.stdout, out.stdout          # rank 0: ECANCELED


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes,ring", [(1500, "1"), (64, "1"), (1500, "0")])
def test_rx_perf_device_resident_from_c(tmp_path, nbytes, ring):
    """examples/rx_perf.c: the device-resident throughput timed from a plain
    C host (the GPU counterpart of iphdr/ipcksumperf.c), its records checked
    against the kept per-packet C APIs (checksums, getters, siphash_buf); the
    device rings from pptk_rx_ring_alloc (default) or plain hipMalloc."""
    exe = build(tmp_path, "rx_perf", hip=True)
    out = subprocess.run([exe, str(1 << 20), str(nbytes), "5"], capture_output=True, text=True,
                         timeout=300, env=dict(os.environ, RX_PERF_RING=ring))
    assert out.returncode == 0, out.stdout + out.stderr
    assert "8192 records checked against the host APIs, 0 mismatches" in out.stdout, out.stdout
    assert ("rings from pptk_rx_ring_alloc" in out.stdout) == (ring == "1"), out.stdout
    print(out.stdout)
