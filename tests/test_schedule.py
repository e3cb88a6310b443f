"""The noise pipeline's schedule, checked on the host (CPU, no GPU).

The reference draws the six noise arrays at the start of each filter() call from one stream whose state carries
across calls (df.cpp:332-349, statics at 334-335; filter() at 449-468). libdfamd generates later calls' noise ahead
of time on a second HIP stream into a ring of noise sets, hands sets over in epochs of `handoff_batch` calls, may run
each epoch's y-passes ahead on a third stream, and restarts the ring when a stream state is loaded, the batch changes
or the batch is restored after 16 calls. None of that may change what any call reads.

A handle created with device = DF_DEVICE_TRACE runs the library's own host logic (df_capi.cpp: gen_begin / gen_end,
consume_gen, prefetch_gen, sweep_ahead, the fused exchange, restart_pipeline) with every HIP call replaced by a
record. From the records this test rebuilds the happens-before order HIP guarantees - program order per stream,
hipStreamWaitEvent binding to the event's latest record enqueued before it, host synchronisation - and checks:
  * every write of a resource (a set's r_ys, r_zs pads, r_zs interior; a stream-state slot; the RNG scratch) is
    ordered after every earlier write of it;
  * every read sees the write it means: the latest write enqueued before it carries the intended generation and
    happens before the read, and every later write happens after the read;
  * every event wait binds to the record it means (or, after a host synchronisation, to nothing still pending).
A deliberately broken schedule (prefetch depth >= the epochs of sets) is caught, so the checker has teeth.
"""
import numpy as np
import pytest

import dfamd

RECORD, WAIT, K1, K3, SHARE, YPASS, PACK, ZPASS, SYNC, STATE_R, STATE_W = range(1, 12)
NSTREAMS = 5  # stream, rng_stream, ystream, comm_stream; 4 = the host


class ScheduleError(AssertionError):
    pass


def accesses(op, a, b, c, d):
    """(resource, tag, is_write) of one record."""
    if op == K1:
        return [(("state", b), a, False), (("scratch",), a, True)]
    if op == K3:
        return [(("scratch",), a, False), (("state", c), a, False), (("ry", b), a, True), (("rzp", b), a, True),
                (("state", d), a + 1, True)]
    if op == SHARE:
        return [(("scratch",), a, True)]
    if op == YPASS:
        return [(("ry", b), a, False), (("rzi", b), a, True)]
    if op == PACK:
        return [(("rzi", b), a, False)]
    if op == ZPASS:
        return [(("rzp", b), a, False), (("rzi", b), a, False)]
    if op == STATE_R:
        return [(("state", a), b, False)]
    if op == STATE_W:
        return [(("state", a), b, True)]
    return []


def check_schedule(tr):
    """Raise ScheduleError on the first hazard or mis-bound wait; return counts of what was checked."""
    last = [np.zeros(NSTREAMS, np.int64) for _ in range(NSTREAMS)]
    count = np.zeros(NSTREAMS, np.int64)
    host = np.zeros(NSTREAMS, np.int64)  # what the host knows complete (syncs) and has done (host ops)
    records = {}  # event -> [(enqueue index, vc, tag, sync count at record)]
    ops = []  # (index, stream, pos, vc)
    per_res = {}  # resource -> [(index, op id, tag, is_write)]
    nsync = 0
    synced_gen = -(1 << 62)  # generations whose every operation was enqueued before the last sync
    max_gen = -(1 << 62)
    nwait = 0
    for i, (op, st, a, b, c, d) in enumerate(tr.tolist()):
        if op == SYNC:
            for s in range(NSTREAMS):
                host = np.maximum(host, last[s])
            nsync += 1
            synced_gen = max_gen
            continue
        s = 4 if op in (STATE_R, STATE_W) else st
        vc = np.maximum(last[s], host)
        count[s] += 1
        vc[s] = count[s]
        if op == WAIT:
            nwait += 1
            bound = None
            for rec in reversed(records.get(a, [])):
                bound = rec
                break
            if bound is not None:
                vc = np.maximum(vc, bound[1])
            if bound is None or bound[2] != b:
                # moot only if what it binds and what it means were both complete at a host sync before it
                moot = (bound is None or bound[3] < nsync) and b <= synced_gen
                if not moot:
                    raise ScheduleError(f"record {i}: wait on event {a} (stream {st}) means generation {b}, "
                                        f"binds to {None if bound is None else bound[2]}")
        elif op == RECORD:
            records.setdefault(a, []).append((i, vc.copy(), b, nsync))
        if s == 4:
            host = np.maximum(host, vc)
        last[s] = vc
        oid = len(ops)
        ops.append((i, s, int(count[s]), vc))
        if op in (K1, K3, SHARE, YPASS, PACK, ZPASS):
            max_gen = max(max_gen, a)
        for res, tag, w in accesses(op, a, b, c, d):
            per_res.setdefault(res, []).append((i, oid, tag, w))

    def hb(x, y):  # op x happens before op y
        _, sx, px, _ = ops[x]
        return ops[y][3][sx] >= px

    nchk = 0
    for res, acc in per_res.items():
        writes = [(i, o, t) for i, o, t, w in acc if w]
        for (i1, o1, t1), (i2, o2, t2) in zip(writes, writes[1:]):
            nchk += 1
            if not hb(o1, o2):  # chained: each write after the one before covers every pair
                raise ScheduleError(f"{res}: write of generation {t2} (record {i2}) not ordered after the write of "
                                    f"generation {t1} (record {i1})")
        latest = None
        for i, o, t, w in acc:
            if w:
                latest = (i, o, t)
                continue
            nchk += 1
            if latest is None or latest[2] != t:
                raise ScheduleError(f"{res}: read of generation {t} (record {i}) follows the write of generation "
                                    f"{None if latest is None else latest[2]}")
            if not hb(latest[1], o):
                raise ScheduleError(f"{res}: read of generation {t} (record {i}) not ordered after its write "
                                    f"(record {latest[0]})")
            nxt = next(((j, p, u) for j, p, u, ww in acc if ww and j > i), None)
            if nxt is not None and not hb(o, nxt[1]):
                raise ScheduleError(f"{res}: write of generation {nxt[2]} (record {nxt[0]}) may run before the read "
                                    f"of generation {t} (record {i})")
    return {"records": len(tr), "waits": nwait, "checks": nchk}


def trace_handle(**kw):
    return dfamd.DigitalFilter(device=dfamd.DEVICE_TRACE, seed=7, **kw)


def run(h, script):
    """script: a list of ("filter", n) | ("load",) | ("hb", v) | ("ahead", v) | ("state",) | ("ghost", v)."""
    for step in script:
        if step[0] == "filter":
            for _ in range(step[1]):
                h.filter(1e-8)
        elif step[0] == "load":
            h.set_rng_state(1234, 0, 0.0)
        elif step[0] == "state":
            h.rng_state()
        elif step[0] == "hb":
            h.set_tuning("handoff_batch", step[1])
        elif step[0] == "ahead":
            h.set_tuning("ypass_ahead", step[1])
        elif step[0] == "ghost":
            h.set_tuning("halo_ghost", step[1])
    return h.trace()


PLANES = {
    "c1": dict(plane="synthetic", Ny=128, Nz=128, N_min=8, N_max=8),
    "c2": dict(plane="synthetic", Ny=512, Nz=512, N_min=4, N_max=32),
    "c3": dict(plane="synthetic", Ny=2048, Nz=2048, N_min=4, N_max=64),
    "native": dict(plane="native"),
}
# calls, state loads (the C++ objects of one process handing the stream on), a read-back, the 16-call restore of
# the hand-off batch after a load, batch changes and y-pass-ahead toggles, mixed
SCRIPT = [("filter", 9), ("state",), ("load",), ("filter", 3), ("load",), ("filter", 20), ("state",), ("filter", 5),
          ("ahead", 1), ("filter", 7), ("load",), ("ahead", 0), ("filter", 19), ("ahead", 1), ("filter", 11),
          ("state",)]
BATCHES = {"c1": (1, 2, 4), "c2": (1, 2), "c3": (1, 2), "native": (1, 2, 4)}


@pytest.mark.parametrize("mode", ["table", "packed"])
@pytest.mark.parametrize("plane", sorted(PLANES))
def test_schedule_of_every_single_gpu_plane(plane, mode):
    h = trace_handle(coeff_mode=mode, **PLANES[plane])
    hb0 = h.get_tuning("handoff_batch")
    script = list(SCRIPT)
    for v in BATCHES[plane]:  # every batch the plane's noise sets allow, then back to its own
        if v != hb0:
            script += [("hb", v), ("filter", 13), ("load",), ("filter", 18)]
    script += [("hb", hb0), ("filter", 10), ("state",)]
    try:
        run(h, script)
    except dfamd.DFError as e:  # a batch this handle's sets cannot hold is refused, nothing else
        assert "noise sets" in str(e), e
    stats = check_schedule(h.trace())
    assert stats["waits"] > 20 and stats["checks"] > 100, stats
    h.close()


@pytest.mark.parametrize("rank", [0, 3, 7])
@pytest.mark.parametrize("ghost", [0, 1])
def test_schedule_of_a_table_zstrip(rank, ghost, monkeypatch):
    # one rank of c4 over 8 in table mode (DFAMD_SOLO_STRIP: the RCCL handle's schedule, the exchange stood in by a
    # copy): generations two calls ahead, share records riding in the halo position, the y-pass ahead
    monkeypatch.setenv("DFAMD_SOLO_STRIP", "1")
    h = trace_handle(coeff_mode="table", plane="synthetic", Ny=256, Nz=8192, N_min=4, N_max=64, rank=rank, world=8)
    assert h.get_tuning("ypass_ahead") == 1
    run(h, [("ghost", ghost), ("filter", 12), ("ahead", 0), ("filter", 5), ("ahead", 1), ("filter", 9),
            ("ghost", 1 - ghost), ("filter", 7)])
    stats = check_schedule(h.trace())
    assert stats["waits"] > 20, stats
    h.close()


def test_checker_catches_a_set_reused_too_early():
    # the hazard of generating as far ahead as the ring is long: two epochs of sets, generation two epochs ahead.
    # Replay the library's own trace with every release wait dropped: generation e + 2 then overwrites sets the
    # z-pass of epoch e may still read
    h = trace_handle(coeff_mode="table", **PLANES["c2"])
    run(h, [("filter", 24)])
    tr = h.trace()
    check_schedule(tr)
    rel = (tr[:, 0] == WAIT) & (tr[:, 2] >= 4) & (tr[:, 2] < 16)
    assert rel.any()
    with pytest.raises(ScheduleError):
        check_schedule(tr[~rel])
    # and a wait bound to the wrong record: the noise-ready waits retargeted one epoch early
    bad = tr.copy()
    ready = (bad[:, 0] == WAIT) & (bad[:, 1] == 0) & (bad[:, 2] < 2)
    bad[ready, 3] -= 1
    with pytest.raises(ScheduleError):
        check_schedule(bad)
    h.close()


def test_trace_handle_is_host_only():
    h = trace_handle(coeff_mode="table", **PLANES["c1"])
    with pytest.raises(dfamd.DFError):
        h.field("u")  # no GPU state behind a trace handle
    h.close()


def test_schedules_cover_every_depth_batch_and_ring():
    # the configurations the runs above check: prefetch depth 1 and 2, hand-off batches 1, 2, 4, rings of 2 and 3
    # epochs of sets (and the 4-set ring of the z-strip's two-calls-ahead generation)
    seen = set()
    for plane in sorted(PLANES):
        for mode in ("table", "packed"):
            h = trace_handle(coeff_mode=mode, **PLANES[plane])
            for v in (h.get_tuning("handoff_batch"),) + BATCHES[plane]:
                try:
                    h.set_tuning("handoff_batch", v)
                except dfamd.DFError:
                    continue
                h.filter(1e-8)
                ns, d = h.get_tuning("noise_sets"), h.get_tuning("prefetch_epochs")
                seen.add((v, ns // v, d))
                check_schedule(h.trace())
            h.close()
    assert {d for _, _, d in seen} == {1, 2}
    assert {v for v, _, _ in seen} == {1, 2, 4}
    assert {(v, k) for v, k, _ in seen} >= {(2, 2), (2, 3), (4, 2), (4, 3)}, seen
    # the re-landed form (round 6): batched single-GPU table planes hold three epochs and generate two ahead
    for plane in ("c1", "c2", "c3"):
        h = trace_handle(coeff_mode="table", **PLANES[plane])
        hb = h.get_tuning("handoff_batch")
        assert hb > 1 and h.get_tuning("noise_sets") == 3 * hb and h.get_tuning("prefetch_epochs") == 2, plane
        h.close()
