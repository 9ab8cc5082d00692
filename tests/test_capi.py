"""The C-ABI library: loads, exports every function include/*.h declares,
and its kept per-packet host APIs give the reference's answers.  No GPU
compute here (CPU suite)."""
import ctypes
import glob
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import framegen
from conftest import ROOT, load_golden

INCLUDE = os.path.join(ROOT, "include")


def _declared_functions():
    names = set()
    for h in glob.glob(os.path.join(INCLUDE, "*.h")):
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        txt = re.sub(r"//[^\n]*", "", txt)
        txt = re.sub(r"#ifdef __cplusplus.*?#endif", "", txt, flags=re.S)
        txt = re.sub(r"#[^\n]*", "", txt)
        depth, cur, stmts = 0, [], []
        for ch in txt:                       # statements at brace depth 0
            if ch == "{":
                depth += 1
                if depth == 1:
                    stmts.append("".join(cur))
                    cur = []
            elif ch == "}":
                depth -= 1
            elif depth == 0:
                if ch == ";":
                    stmts.append("".join(cur))
                    cur = []
                else:
                    cur.append(ch)
        for stmt in stmts:
            stmt = " ".join(stmt.split())
            m = re.match(r"^((?:const )?(?:struct )?\w[\w \*]*?)\b(\w+) ?\(([^()]*)\)$", stmt)
            if not m or "static" in m.group(1) or "typedef" in m.group(1):
                continue
            names.add(m.group(2))
    return names


@pytest.fixture(scope="module")
def lib():
    from pptk_amd import rx
    return rx.lib()


def test_library_exports_every_declared_function(lib):
    declared = _declared_functions()
    assert {"pptk_rx_batch", "pptk_rx_batch_device", "ip_cksum_feed",
            "tcp6_cksum_calc", "hash_seed_init"} <= declared
    missing = [f for f in sorted(declared) if not hasattr(lib, f)]
    assert not missing, missing
    for var in ("hash_seed", "hash_seed_inited"):
        assert ctypes.c_int.in_dll(lib, var) is not None


def test_exports_list_matches(lib):
    from pptk_amd import rx
    assert set(rx.EXPORTS) <= _declared_functions()


def test_host_ip_cksum_feed_matches_oracle(lib, oracle_lib):
    rng = np.random.default_rng(11)
    for n in list(range(0, 80)) + [255, 1024, 1499, 1500, 9000, 65535]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        s = ctypes.c_uint32(0)
        lib.ip_cksum_feed(ctypes.byref(s), data, n)
        post = s.value
        while post >> 16:
            post = (post & 0xFFFF) + (post >> 16)
        got = ((~post & 0xFFFF) >> 8) | (((~post) & 0xFF) << 8)
        assert got == oracle_lib.cksum(data), n
    # all-zero input: 0xffff in both
    s = ctypes.c_uint32(0)
    lib.ip_cksum_feed(ctypes.byref(s), bytes(100), 100)
    assert s.value == 0


@pytest.mark.parametrize("name", ["edge", "cmix", "fuzz"])
def test_host_l4_cksums_match_golden(lib, name):
    """tcp/udp(6)_cksum_calc from libpptkrx.so reproduce the golden l4_cksum
    of every frame that has an L4 header."""
    from pptk_amd.records import F_IPV6, F_L4, as_records
    z = load_golden(name)
    recs = as_records(z["recs"])
    buf = z["buf"]
    n_checked = 0
    for i in np.nonzero(recs["flags"] & F_L4)[0]:
        r = recs[i]
        o = int(z["off"][i])
        f = buf[o:o + int(z["len"][i])].tobytes()
        ip = f[r["l3_off"]:]
        l4 = f[r["l4_off"]:]
        v6 = bool(r["flags"] & F_IPV6)
        fn = {(6, False): lib.tcp_cksum_calc, (17, False): lib.udp_cksum_calc,
              (6, True): lib.tcp6_cksum_calc, (17, True): lib.udp6_cksum_calc}[(int(r["proto"]), v6)]
        iplen = 40 if v6 else (ip[0] & 15) * 4
        assert fn(ip, iplen, l4, int(r["l4_len"])) == r["l4_cksum"], i
        if not v6:
            assert lib.ip_hdr_cksum_calc(ip, iplen) == r["ip_cksum"]
        n_checked += 1
    assert n_checked > 100


def test_c_dropin_program(tmp_path):
    """Compile a C client with plain gcc against include/ + libpptkrx.so."""
    exe = str(tmp_path / "capi_dropin")
    libdir = os.path.join(ROOT, "pptk_amd")
    subprocess.check_call(["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-Werror",
                           "-I", INCLUDE, os.path.join(ROOT, "tests", "c", "capi_dropin.c"),
                           "-L", libdir, "-lpptkrx", f"-Wl,-rpath,{libdir}", "-o", exe])
    import torch
    args = [exe] + ([] if torch.cuda.is_available() else ["nogpu"])
    out = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "capi_dropin ok" in out.stdout


@pytest.mark.parametrize("struct,dtname", [("pptk_rx_rec", "REC_DTYPE"),
                                            ("pptk_rx_rec32", "REC32_DTYPE"),
                                            ("pptk_rx_frag", "FRAG_DTYPE")])
def test_record_layout_matches_header(struct, dtname):
    import pptk_amd.records as R
    dt = getattr(R, dtname)
    txt = open(os.path.join(INCLUDE, "pptk_rx.h")).read()
    body = txt[txt.index(f"struct {struct} {{"):]
    body = body[:body.index("};")]
    for name in dt.names:
        off = dt.fields[name][1]
        m = re.search(rf"\b{name}(\[\d+\])?;\s*/\*\s*(\d+)", body)
        assert m and int(m.group(2)) == off, name


def test_bench_and_tools_compile():
    """bench.py and the tooling must at least compile on CPU (the GPU box's
    interpreter rejects what the local parser might let through)."""
    import py_compile
    for f in ("bench.py", "__graft_entry__.py", "tools/ab.py", "tools/e2e.py",
              "harness/membench.py", "harness/synth.py", "harness/rwmix.py", "tools/pmc_summary.py",
              "tools/permit_run.py", "tools/permit_pmc.py"):
        py_compile.compile(os.path.join(ROOT, f), doraise=True)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "--steps" in out.stdout


def _build_rx_loop(tmp_path):
    exe = str(tmp_path / "rx_loop")
    libdir = os.path.join(ROOT, "pptk_amd")
    subprocess.check_call(["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-Werror",
                           "-I", INCLUDE, os.path.join(ROOT, "examples", "rx_loop.c"),
                           "-L", libdir, "-lpptkrx", f"-Wl,-rpath,{libdir}", "-o", exe])
    return exe


def test_example_rx_loop_builds(tmp_path):
    """examples/rx_loop.c (the INTEGRATION.md walk-through) builds with gcc."""
    _build_rx_loop(tmp_path)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [[], ["pipe"]])
def test_example_rx_loop_runs(tmp_path, mode):
    """The LDP-style rx loop verifies every frame but the one it corrupted,
    synchronous and pipelined (pptk_rx_batch_submit / _complete)."""
    out = subprocess.run([_build_rx_loop(tmp_path), "20"] + mode, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "20000 frames" in out.stdout and "19995 verified, 5 failed" in out.stdout


@pytest.fixture(scope="module")
def kept_inline(tmp_path_factory):
    """tests/c/kept_inline.c: the kept inline setters / incremental updates
    of include/ipcksum.h wrapped as exported functions (built with gcc)."""
    import ctypes
    so = str(tmp_path_factory.mktemp("kept") / "libkept.so")
    libdir = os.path.join(ROOT, "pptk_amd")
    subprocess.check_call(["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-Werror", "-fPIC",
                           "-shared", "-I", INCLUDE, os.path.join(ROOT, "tests", "c", "kept_inline.c"),
                           "-L", libdir, "-lpptkrx", f"-Wl,-rpath,{libdir}", "-o", so])
    L = ctypes.CDLL(so)
    u16, u32, vp = ctypes.c_uint16, ctypes.c_uint32, ctypes.c_void_p
    L.kept_update16.argtypes, L.kept_update16.restype = [u16, u16, u16], u16
    L.kept_update32.argtypes, L.kept_update32.restype = [u16, u32, u32], u16
    L.kept_rewrite.argtypes = [vp] + [ctypes.c_int] * 4 + [u32, u32, u32, u16, u16,
                                                         ctypes.c_int, ctypes.c_int]
    L.kept_set_cksums.argtypes = [vp] + [ctypes.c_int] * 5 + [u16]
    L.kept_set_cksums.restype = None
    return L


def test_kept_update_helpers(kept_inline, oracle_lib):
    rng = np.random.default_rng(3)
    for _ in range(20000):
        c, a, b = (int(x) for x in rng.integers(0, 65536, 3))
        assert kept_inline.kept_update16(c, a, b) == oracle_lib.update_cksum16(c, a, b)
        a32, b32 = (int(x) for x in rng.integers(0, 2 ** 32, 2))
        assert kept_inline.kept_update32(c, a32, b32) == oracle_lib.update_cksum32(c, a32, b32)


def test_kept_update_helpers_vs_reference(kept_inline, reference_lib):
    rng = np.random.default_rng(4)
    for _ in range(20000):
        c, a, b = (int(x) for x in rng.integers(0, 65536, 3))
        assert kept_inline.kept_update16(c, a, b) == reference_lib.update_cksum16(c, a, b)


@pytest.mark.parametrize("tag,name", [("edge", "edge"), ("fuzz", "fuzz"), ("cmix", "cmix"),
                                      ("icmp", "icmp")])
def test_kept_rewrite_functions_match_fixture(kept_inline, tag, name):
    """The kept per-frame *_cksum_update functions, applied frame by frame
    as pptk_tx_rewrite_device composes them, give the reference's bytes."""
    import ctypes
    from pptk_amd.records import (F_FRAGMENT, F_L4, F_PARSED, RW_ST_TTL_ZERO, as_records)
    from test_oracle import rewrite_case
    z, buf_in, buf_out, rw, status = rewrite_case(tag, name)
    recs = as_records(z["recs"])
    buf = buf_in.copy()
    n_done = 0
    for i, o in enumerate(z["off"]):
        if status[i] == 0 or status[i] & RW_ST_TTL_ZERO:
            continue
        r, w = recs[i], rw[i]
        L = int(z["len"][i])
        fr = (ctypes.c_uint8 * L).from_buffer(buf, int(o))
        kept_inline.kept_rewrite(fr, int(r["l3_off"]), int(r["l4_off"]), int(r["proto"]),
                                 int(bool(r["flags"] & F_L4)), int(w["ops"]), int(w["src"]),
                                 int(w["dst"]), int(w["sport"]), int(w["dport"]),
                                 int(r["l4_len"]), int(bool(r["flags"] & F_FRAGMENT)))
        assert r["flags"] & F_PARSED
        n_done += 1
    assert n_done > 50
    assert np.array_equal(buf, buf_out), int((buf != buf_out).sum())


@pytest.mark.parametrize("name", ["edge", "fuzz", "cmix"])
def test_kept_tx_setters_match_fixture(kept_inline, name):
    import ctypes
    from pptk_amd.records import F_IPV6, F_L4, F_MALFORMED, F_PARSED, as_records
    z = load_golden(name)
    t = load_golden("tx")
    pos = t[f"{name}_pos"].astype(np.int64)
    buf = z["buf"].copy()
    buf[pos] = t[f"{name}_in"]
    want = buf.copy()
    want[pos] = t[f"{name}_out"]
    recs = as_records(z["recs"])
    for i, o in enumerate(z["off"]):
        r = recs[i]
        fl = int(r["flags"])
        if not fl & F_PARSED or fl & F_MALFORMED:
            continue
        L = int(z["len"][i])
        fr = (ctypes.c_uint8 * L).from_buffer(buf, int(o))
        kept_inline.kept_set_cksums(fr, int(r["l3_off"]), int(r["l4_off"]), int(bool(fl & F_IPV6)),
                                    int(r["proto"]), int(bool(fl & F_L4)), int(r["l4_len"]))
    assert np.array_equal(buf, want), int((buf != want).sum())


# ---- kept TCP option API (include/iphdr.h walks, include/ipcksum.h option
# rewrites) vs the reference's results in tests/golden/tcpopt.npz
def _kept_tcpopt(kept_inline):
    L = kept_inline
    vp = ctypes.c_void_p
    L.kept_tcp_parse_options.restype = ctypes.c_uint32
    L.kept_tcp_parse_options.argtypes = [vp, vp, vp, vp]
    L.kept_tcp_find_sack_ts.restype = ctypes.c_uint32
    L.kept_tcp_find_sack_ts.argtypes = [vp]
    L.kept_tcp_find_sack.restype = ctypes.c_int64
    L.kept_tcp_find_sack.argtypes = [vp, vp, vp]
    L.kept_tcp_opt_op.restype = None
    L.kept_tcp_opt_op.argtypes = [vp, ctypes.c_int, ctypes.c_uint32]
    return L


def test_kept_tcp_option_walks_match_fixture(kept_inline):
    L = _kept_tcpopt(kept_inline)
    z = load_golden("tcpopt")
    for i, h0 in enumerate(z["hdrs"]):
        h = np.ascontiguousarray(h0).copy()
        p = h.ctypes.data_as(ctypes.c_void_p)
        mss, ts, te = ctypes.c_uint16(), ctypes.c_uint32(), ctypes.c_uint32()
        got = L.kept_tcp_parse_options(p, ctypes.byref(mss), ctypes.byref(ts), ctypes.byref(te))
        assert [got, mss.value, ts.value, te.value] == list(z["parse"][i]), i
        if z["sackts"][i, 1]:                  # the reference returned on this input
            assert L.kept_tcp_find_sack_ts(p) == z["sackts"][i, 0], i
        sl, al = ctypes.c_uint32(), ctypes.c_int()
        off = L.kept_tcp_find_sack(p, ctypes.byref(sl), ctypes.byref(al))
        assert [off, sl.value, al.value] == list(z["sack"][i]), i
        assert np.array_equal(h, h0)           # the walks never write


def test_kept_tcp_option_rewrites_match_fixture(kept_inline):
    L = _kept_tcpopt(kept_inline)
    z = load_golden("tcpopt")
    ran = 0
    for i, h0 in enumerate(z["hdrs"]):
        op, val, ok = (int(x) for x in z["ops"][i])
        if not ok:                             # the reference never returns here
            continue
        h = np.ascontiguousarray(h0).copy()
        L.kept_tcp_opt_op(h.ctypes.data_as(ctypes.c_void_p), op, val)
        assert np.array_equal(h, z["after"][i]), (i, op)
        ran += 1
    assert ran > 2900


def test_kept_tcp_option_api_vs_reference(kept_inline, reference_lib):
    """Fresh headers (another seed) against live reference calls."""
    L = _kept_tcpopt(kept_inline)
    R = reference_lib.lib
    hdrs = framegen.tcp_headers(2000, seed=0xBEE)
    rng = np.random.default_rng(5)
    for h0 in hdrs:
        term, so, sl, _ = framegen.sack_ts_walk(h0)
        a, b = h0.copy(), h0.copy()
        pa, pb = a.ctypes.data_as(ctypes.c_void_p), b.ctypes.data_as(ctypes.c_void_p)
        m1, m2 = ctypes.c_uint16(), ctypes.c_uint16()
        t1, t2, e1, e2 = (ctypes.c_uint32() for _ in range(4))
        assert L.kept_tcp_parse_options(pa, ctypes.byref(m1), ctypes.byref(t1),
                                        ctypes.byref(e1)) == \
            R.ref_tcp_parse_options(pb, ctypes.byref(m2), ctypes.byref(t2), ctypes.byref(e2))
        assert (m1.value, t1.value, e1.value) == (m2.value, t2.value, e2.value)
        if term:
            assert L.kept_tcp_find_sack_ts(pa) == R.ref_tcp_find_sack_ts(pb)
        for op in range(9):
            if op in (2, 3, 4) and (not term or (op == 2 and so % 2 == 1 and sl >= 10)):
                continue
            v = int(rng.integers(0, 2 ** 32))
            L.kept_tcp_opt_op(pa, op, v)
            R.ref_tcp_opt_op(pb, op, v)
            assert np.array_equal(a, b), op


def test_kept_tcp_find_sack_ts_stops_where_reference_loops(kept_inline):
    """A SACK option with length byte 0: the reference's walk never returns
    (iphdr/iphdr.c:152-163 adds 0); the kept walk stops there with the SACK
    option recorded."""
    L = _kept_tcpopt(kept_inline)
    h = np.zeros(80, np.uint8)
    h[12] = 8 << 4                              # 32-byte header, 12 bytes of options
    h[20:24] = [1, 1, 5, 0]
    assert not framegen.sack_ts_walk(h)[0]
    assert L.kept_tcp_find_sack_ts(h.ctypes.data_as(ctypes.c_void_p)) == 22 | (0 << 8)


# ---- kept rate limiter (include/iphash.h) and timer heap (include/timerlink.h)
def _build_iphash_harness(out, reference=False):
    """tests/c/iphash_scenario.c against the kept API (include/ +
    libpptkrx.so) or, reference=True, against the reference's own headers and
    objects in oracle/_ref (built from /root/reference)."""
    src = os.path.join(ROOT, "tests", "c", "iphash_scenario.c")
    if not reference:
        libdir = os.path.join(ROOT, "pptk_amd")
        cmd = ["gcc", "-O2", "-std=gnu11", "-Wall", "-Werror", "-fPIC", "-shared", "-I", INCLUDE,
               src, "-L", libdir, "-lpptkrx", f"-Wl,-rpath,{libdir}", "-o", out]
    else:
        from oracle.oracle import REF_SO
        ref, obj = "/root/reference", os.path.join(os.path.dirname(REF_SO), "obj")
        incs = [f"-I{ref}/{d}" for d in ("iphash", "timerlinkheap", "misc", "hashtable", "log",
                                           "hashlist", "linkedlist")]
        objs = [os.path.join(obj, p) for p in ("iphash/iphash.o", "timerlinkheap/timerlink.o",
                                               "misc/hashseed.o", "log/log.o")]
        cmd = ["gcc", "-O2", "-std=gnu11", "-fPIC", "-shared", *incs, src, *objs, "-pthread",
               "-o", out]
    subprocess.check_call(cmd)
    L = ctypes.CDLL(out)
    vp, u32, u8, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_size_t
    L.iphash_scenario.restype = u32
    L.iphash_scenario.argtypes = [vp, ctypes.c_int, u8, vp, vp, sz, u32, u32, u32, u32, u32, sz,
                                  vp, vp]
    L.iphash_permit_seq.restype = None
    L.iphash_permit_seq.argtypes = [vp, ctypes.c_int, u8, vp, vp, vp, sz, u32, u32, vp, vp, vp]
    L.timer_heap_exercise.restype = ctypes.c_long
    L.timer_heap_exercise.argtypes = [ctypes.c_uint64, sz, sz, vp, sz]
    return L


@pytest.fixture(scope="module")
def iphash_kept(tmp_path_factory):
    return _build_iphash_harness(str(tmp_path_factory.mktemp("iph") / "kept.so"))


@pytest.fixture(scope="module")
def iphash_ref(tmp_path_factory):
    from oracle.oracle import REF_SO
    if not os.path.exists(REF_SO) or not os.path.isdir("/root/reference/iphash"):
        pytest.skip("reference tree / oracle/_ref absent")
    return _build_iphash_harness(str(tmp_path_factory.mktemp("iphr") / "ref.so"), True)


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _sources(recs):
    from pptk_amd.records import F_IPV6, F_PARSED, as_records
    r = as_records(recs)
    src4 = np.ascontiguousarray(r["src"][:, :4].astype(np.uint32) @ np.array([1 << 24, 1 << 16, 1 << 8, 1],
                                                                               np.uint32))
    src6 = np.ascontiguousarray(r["src"])
    parsed = (r["flags"] & F_PARSED) != 0
    v6 = (r["flags"] & F_IPV6) != 0
    return src4.astype(np.uint32), src6, parsed, v6


def test_kept_iphash_matches_permit_fixture(iphash_kept):
    """ip_permitted / ipv6_permitted of the kept API, once per frame in frame
    order, give the reference's verdicts and token arrays
    (tests/golden/permit.npz, made with the reference's own functions)."""
    z = load_golden("permit")
    bits4, bits6, hs = (int(x) for x in z["iphash"])
    src4, src6, parsed, v6 = _sources(z["recs"])
    key = np.ascontiguousarray(z["key"])
    for k, (fam, init, has_subj) in enumerate(z["case_meta"]):
        use = (parsed & (v6 == (fam == 6))).astype(np.uint8)
        if has_subj:
            use &= z["case_subject"][k].astype(np.uint8)
        verdict = np.zeros(len(use), np.uint8)
        tok_in = np.ascontiguousarray(z["case_tok_in"][k].astype(np.uint32))
        tok = np.zeros(hs, np.uint32)
        iphash_kept.iphash_permit_seq(_p(key), int(fam), bits4 if fam == 4 else bits6, _p(src4),
                                      _p(src6), _p(use), len(use), hs, int(init), _p(tok_in),
                                      _p(verdict), _p(tok))
        assert np.array_equal(verdict, z["case_verdict"][k]), (fam, init)
        assert np.array_equal(tok, z["case_tok_out"][k]), (fam, init)


@pytest.mark.parametrize("family,bits", [(4, 24), (4, 32), (6, 48), (6, 128)])
@pytest.mark.parametrize("initial", [3, 200, 1000, 70000])
def test_kept_iphash_timer_scenario_vs_reference(iphash_kept, iphash_ref, family, bits, initial):
    """The same timer-driven scenario (permits, give-backs, refill timers
    fired from the heap by a virtual clock) against the reference build:
    verdicts, final tokens and the number of timer firings agree."""
    rng = np.random.default_rng(family * 1000 + bits + initial)
    n = 20000
    prefixes = rng.integers(0, 2 ** 32, 5, dtype=np.uint64).astype(np.uint32)
    src4 = np.ascontiguousarray(prefixes[rng.integers(0, 5, n)] ^
                                rng.integers(0, 256, n).astype(np.uint32))
    src6 = np.ascontiguousarray(rng.integers(0, 256, (n, 16), dtype=np.uint8))
    src6[:, :6] = rng.integers(0, 256, (5, 6), dtype=np.uint8)[rng.integers(0, 5, n)]
    key = np.arange(1, 17, dtype=np.uint8)
    out = []
    for L in (iphash_kept, iphash_ref):
        verdict = np.zeros(n, np.uint8)
        tok = np.zeros(256, np.uint32)
        fired = L.iphash_scenario(_p(key), family, bits, _p(src4), _p(src6), n, 256, 32, initial,
                                  max(1, initial // 4), 9000, 500, _p(verdict), _p(tok))
        out.append((verdict, tok, fired))
    assert out[0][2] == out[1][2] and out[0][2] > 8
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
    assert (out[0][0] == 1).any()
    if initial <= 200 and bits not in (32, 128):    # prefixes share buckets: demand outruns refills
        assert (out[0][0] == 0).any()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_kept_timer_heap(iphash_kept, seed):
    """Random add / modify / remove sequences: pops come out in time order
    and every timer left in the heap comes out."""
    outs = np.zeros(5000, np.uint64)
    n = iphash_kept.timer_heap_exercise(seed, 4000, 200000, _p(outs), len(outs))
    assert n > 1000
    assert np.all(np.diff(outs[:min(n, len(outs))].astype(np.int64)) >= 0)


def test_kept_timer_heap_same_pops_as_reference(iphash_kept, iphash_ref):
    """The same operation sequence on the reference's heap pops the same
    multiset of times in the same (non-decreasing) order."""
    a, b = np.zeros(5000, np.uint64), np.zeros(5000, np.uint64)
    na = iphash_kept.timer_heap_exercise(7, 3000, 100000, _p(a), len(a))
    nb = iphash_ref.timer_heap_exercise(7, 3000, 100000, _p(b), len(b))
    assert na == nb and np.array_equal(a, b)


def test_entry_points_reject_bad_arguments(lib):
    """Every C-ABI entry point answers a null context or contract-violating
    arguments with -EINVAL before touching the GPU (include/pptk_rx.h error
    conventions: 0 or -errno, never an abort)."""
    from pptk_amd.rx import RxDevBatch, RxOpts
    EINVAL = -22
    vp = ctypes.c_void_p
    assert lib.pptk_rx_ctx_create(None, None) == EINVAL
    out = vp()
    bad = RxOpts()
    lib.pptk_rx_opts_default(ctypes.byref(bad))
    bad.iphash_bits4 = 33
    assert lib.pptk_rx_ctx_create(ctypes.byref(out), ctypes.byref(bad)) == EINVAL
    bad.iphash_bits4, bad.iphash_size = 24, 1000          # not a power of two
    assert lib.pptk_rx_ctx_create(ctypes.byref(out), ctypes.byref(bad)) == EINVAL
    assert lib.pptk_rx_batch(None, None, 1, None) == EINVAL
    assert lib.pptk_rx_batch_submit(None, None, 1, None) == EINVAL
    assert lib.pptk_rx_batch32(None, None, 1, None) == EINVAL
    assert lib.pptk_rx_batch_submit32(None, None, 1, None) == EINVAL
    assert lib.pptk_rx_batch_complete(None) == EINVAL
    assert lib.pptk_rx_batch_pending(None) == EINVAL
    b = RxDevBatch()
    assert lib.pptk_rx_batch_device(None, ctypes.byref(b), None) == EINVAL
    assert lib.pptk_rx_batch_device_mixed(None, ctypes.byref(b), None, None, None) == EINVAL
    assert lib.pptk_tx_cksum_device(None, None, None, None, 0, 0, 1, 0, None) == EINVAL
    assert lib.pptk_tx_rewrite_device(None, None, None, None, 0, 0, 1, None, 1, None, None) == EINVAL
    assert lib.pptk_tcp_mss_clamp_device(None, None, None, None, 0, 0, 1, 1460, 0, None, None) == EINVAL
    assert lib.pptk_rx_permit_device(None, None, None, 1, 4, None, None, None, None, None) == EINVAL
    assert lib.pptk_rx_tokens_refill_device(None, None, 0, 1, 1, 1, None) == EINVAL
    assert lib.pptk_rx_bin_device(None, None, 1, None, None, None) == EINVAL
    assert lib.pptk_rx_set_tuning(None, 0, 0) == EINVAL
    assert lib.pptk_rx_register_ring(None, None, 0) == EINVAL
    assert lib.pptk_rx_unregister_ring(None, None) == EINVAL
    assert lib.pptk_rx_last_variant(None) == -1
    # multi-GPU part (include/pptk_rx.h "Multi-GPU")
    uid = ctypes.create_string_buffer(128)
    assert lib.pptk_rx_comm_uid(None) == EINVAL
    assert lib.pptk_rx_comm_create(None, 1, 0, uid) == EINVAL
    assert lib.pptk_rx_comm_create_all(None, 1) == EINVAL
    nul = (vp * 2)(None, None)
    assert lib.pptk_rx_comm_create_all(nul, 2) == EINVAL
    assert lib.pptk_rx_comm_create_all(nul, 0) == EINVAL
    assert lib.pptk_rx_comm_destroy(None) == EINVAL
    assert lib.pptk_rx_comm_info(None, None, None) == EINVAL
    assert lib.pptk_rx_allgather_hash(None, None, 1, None, None) == EINVAL
    assert lib.pptk_rx_stream_split(None, 32, None, None) == EINVAL
    assert lib.pptk_rx_stream_destroy(None) == EINVAL
    assert lib.pptk_rx_stream_split(None, 0, None, None) == EINVAL
    assert lib.pptk_rx_stream_split(None, -1, None, None) == EINVAL
    assert lib.pptk_rx_place_records(None, ctypes.byref(b), None, 1, 1, None, None, None) == EINVAL
    assert lib.pptk_rx_place_buffers(None, ctypes.byref(b), None, 1, None, 1, 1, None, None, None,
                                     None) == EINVAL
    from pptk_amd.rx import RxRingC, RxRingSpec
    spec, ring = RxRingSpec(1 << 20, 16, 64), RxRingC()
    assert lib.pptk_rx_ring_alloc(None, ctypes.byref(spec), ctypes.byref(ring), None) == EINVAL
    assert lib.pptk_rx_ring_free(None) == EINVAL
    assert lib.pptk_rx_ring_free(ctypes.byref(ring)) == 0   # an empty ring: nothing to free
    from pptk_amd.rx import RxGatherC, RxGatherSpec
    gs, g = RxGatherSpec(16, 1, 0), RxGatherC()
    assert lib.pptk_rx_gather_alloc(None, ctypes.byref(b), ctypes.byref(gs), ctypes.byref(g),
                                    None) == EINVAL
    assert lib.pptk_rx_gather_free(None) == EINVAL
    assert lib.pptk_rx_gather_free(ctypes.byref(g)) == 0    # empty: nothing to free
    assert lib.pptk_rx_permit_status(None, None, None) == EINVAL
    lib.pptk_rx_ctx_destroy(None)                           # a no-op


def test_host_sources_under_sanitizers(tmp_path):
    """tests/c/host_fuzz.c built with AddressSanitizer + UBSan (and
    LeakSanitizer at exit) directly from pptk_amd/csrc/host/*.c: random and
    malformed TCP option lists in exactly-sized heap blocks, every
    incremental checksum update keeping the packet verifying, the checksum
    feed against a byte-wise sum, timer-heap invariants and ip_hash
    lifetimes.  Host code only -- GPU sanitizers are not available."""
    exe = str(tmp_path / "host_fuzz")
    srcs = sorted(glob.glob(os.path.join(ROOT, "pptk_amd", "csrc", "host", "*.c")))
    subprocess.check_call(["gcc", "-O1", "-g", "-std=gnu11", "-Wall", "-Wextra", "-Werror",
                           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                           "-I", INCLUDE, os.path.join(ROOT, "tests", "c", "host_fuzz.c"),
                           *srcs, "-pthread", "-o", exe])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    for seed in (1, 2, 3):
        out = subprocess.run([exe, str(seed), "8000"], capture_output=True, text=True,
                             timeout=120, env=env)
        assert out.returncode == 0, out.stdout + out.stderr[-4000:]
        assert "host_fuzz ok" in out.stdout


def test_permit_pmc_summary(tmp_path):
    """tools/permit_pmc.py: per-kernel medians of rocprofv3 counter CSVs,
    FETCH_SIZE doubled (KiB -> MB), the call's total."""
    import csv
    sys.path.insert(0, ROOT)
    from tools import permit_pmc
    for cname, vals in (("FETCH_SIZE", [1000.0, 1200.0, 1100.0]), ("WRITE_SIZE", [500.0] * 3)):
        d = tmp_path / f"pmc_keys_{cname}"
        d.mkdir()
        with open(d / "run_counter_collection.csv", "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            for i, v in enumerate(vals):
                w.writerow([i, "void pptk::(anonymous namespace)::permit_fused<true>(x)", cname, v / 2])
                w.writerow([i, "void pptk::(anonymous namespace)::permit_fused<true>(x)", cname, v / 2])
                w.writerow([i, "rx_kernel", cname, 99999.0])
    fe = permit_pmc.per_kernel(str(tmp_path / "pmc_keys_FETCH_SIZE"), "FETCH_SIZE")
    assert list(fe) == ["permit_fused"] and abs(fe["permit_fused"] - 1100 * 1024 / 1e6) < 1e-9


def test_ctypes_structs_match_the_header(tmp_path):
    """The ctypes mirrors of the C-ABI's structs (pptk_amd/rx.py) have the
    size and field offsets gcc gives the header's structs."""
    from pptk_amd import rx as R
    structs = {"pptk_rx_opts": R.RxOpts, "pptk_rx_dev_batch": R.RxDevBatch,
               "pptk_rx_ring_spec": R.RxRingSpec, "pptk_rx_ring": R.RxRingC,
               "pptk_rx_gather_spec": R.RxGatherSpec, "pptk_rx_gather": R.RxGatherC}
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "pptk_rx.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} sizeof %zu\\n", sizeof(struct {cname}));')
        for fname, _ in py._fields_:
            lines.append(f'  printf("{cname} {fname} %zu\\n", offsetof(struct {cname}, {fname}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = str(tmp_path / "layout")
    subprocess.check_call(["gcc", "-std=gnu11", "-Wall", "-Werror", "-I", INCLUDE, str(src), "-o", exe])
    got = {}
    for line in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.splitlines():
        c, f, v = line.split()
        got[(c, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)


def test_comm_config_caps_channels_only_when_split():
    """The communicator configuration the library builds (rx_comm.hip
    comm_config, through the test library's hook; no GPU): non-blocking
    always; ncclConfig_t.maxCTAs = the CUs pptk_rx_stream_split left the
    collective when the context is split, RCCL's default (unset) when not.
    bench.py sets no NCCL_* variable for this any more."""
    from conftest import HOOKS_LIB
    L = ctypes.CDLL(HOOKS_LIB)
    f = L.pptk_rx_test_comm_config
    f.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_int)] * 3
    undef = -(1 << 31)                                  # NCCL_CONFIG_UNDEF_INT
    for cus, want_max in ((0, undef), (32, 32), (64, 64), (128, 128)):
        b, mn, mx = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        assert f(cus, ctypes.byref(b), ctypes.byref(mn), ctypes.byref(mx)) == 0
        assert (b.value, mn.value, mx.value) == (0, undef, want_max), cus
    assert "NCCL_MAX_NCHANNELS" not in open(os.path.join(ROOT, "bench.py")).read()
    # the product library has no such hook
    assert not hasattr(ctypes.CDLL(os.path.join(ROOT, "pptk_amd", "libpptkrx.so")),
                       "pptk_rx_test_comm_config")


def test_abi_revision_matches_header(lib):
    """pptk_rx_abi() == the header's PPTK_RX_ABI == the Python binding's:
    a caller can detect a library whose structs differ from its header."""
    from pptk_amd import rx as R
    txt = open(os.path.join(INCLUDE, "pptk_rx.h")).read()
    hdr = int(re.search(r"#define PPTK_RX_ABI (\d+)", txt).group(1))
    assert lib.pptk_rx_abi() == hdr == R.ABI
