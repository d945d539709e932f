"""Per-kernel timing of the training step inside the captured HIP graphs
(libngp_amd.so's ngp_timing_set hook: every instrumented launch is
bracketed by two one-lane kernels that store the GPU wall clock into a
stamp table on the device, row = the trainer's device step counter, so a
replayed graph times every one of its kernels; HIP event nodes inside
captured graphs are not available with the HIP runtime torch ships).

A stamp pair measures from the end of the kernel before the launch (the
stamp kernel runs when its predecessor in the stream has finished) to the
end of the launch: the kernel's execution plus its dispatch gap, like a HIP
event pair around it.  Measurement plumbing only (bench.py, scripts/); the
product path never arms it."""
from __future__ import annotations

import ctypes
import itertools
from ctypes import c_int32

import torch

import vren

NAMES = ["sample_batch", "bitfield_summary", "march", "scan_rays", "march_compact", "segments", "hash_encode",
         "field_mlp", "chunk_rest", "composite_loss", "hash_count", "hash_scan", "hash_plan", "mlp_bwd",
         "hash_bwd_coarse", "hash_write", "hash_accum", "adam"]  # include/ngp_amd.h NGP_K_* order
_UID = itertools.count(1)
PER_ID = 8  # launches per kernel id per step (segments: one per evaluation round + 1, encode / MLP: one per round, +1 in occupancy updates)


def _lib():
    return vren.lib()  # signatures declared in vren._declare


class KernelTimer:
    """Stamp table for `rows` steps (row = step counter % rows) of the kernels
    `names` (None: all).  trainer.timer = KernelTimer(...) makes NGPTrainer
    capture (and replay) graphs with the stamps inside; read() after a
    synchronize returns per-launch durations of every step that ran.
    span=(first, last): only a stamp before `first` and one after `last`
    (consecutive launches on one stream timed together: read_span())."""

    def __init__(self, step_counter, rows=4096, names=None, device="cuda", span=None):
        self.step = step_counter  # int64 device scalar: the row of the running step
        self.rows = rows
        self.row_len = len(NAMES) * PER_ID * 2
        self.stamps = torch.zeros(rows, self.row_len, dtype=torch.int64, device=device)
        ids = range(len(NAMES)) if names is None else [NAMES.index(n) for n in names]
        self.begin_mask = self.end_mask = sum(1 << i for i in ids)
        self.span = span
        if span is not None:
            self.begin_mask, self.end_mask = 1 << NAMES.index(span[0]), 1 << NAMES.index(span[1])
        self.tick_ns = _lib().ngp_timing_tick_ns()
        self.uid = next(_UID)  # graphs captured with this table are keyed by it (never reused)

    def arm(self):
        vren._ok(_lib().ngp_timing_set(self.stamps.data_ptr(), self.step.data_ptr(), self.rows, len(NAMES), PER_ID,
                                       self.begin_mask, self.end_mask), "timing_set")

    def disarm(self):
        """-> launches per kernel id bracketed since arm()"""
        c = (c_int32 * len(NAMES))()
        vren._ok(_lib().ngp_timing_counts(c, len(NAMES)), "timing_counts")
        vren._ok(_lib().ngp_timing_set(None, None, 0, 0, 0, 0, 0), "timing_set")
        return list(c)

    def reset(self):
        self.stamps.zero_()

    def read(self):
        """{kernel: [ms per launch, ...]} over the rows written since reset()"""
        st = self.stamps.cpu().view(self.rows, len(NAMES), PER_ID, 2)
        a, b = st[..., 0], st[..., 1]
        ok = (a > 0) & (b >= a)
        ms = (b - a).double() * self.tick_ns * 1e-6
        out = {}
        for k, n in enumerate(NAMES):
            m = ok[:, k, :]
            if m.any():
                out[n] = ms[:, k, :][m].tolist()
        return out

    def read_span(self):
        """[ms per step] from the stamp before span[0]'s first launch to the
        one after span[1]'s first launch, over the rows written"""
        st = self.stamps.cpu().view(self.rows, len(NAMES), PER_ID, 2)
        a = st[:, NAMES.index(self.span[0]), 0, 0]
        b = st[:, NAMES.index(self.span[1]), 0, 1]
        ok = (a > 0) & (b >= a)
        return ((b - a)[ok].double() * self.tick_ns * 1e-6).tolist()

    def timeline(self):
        """{"kernel#slot": (avg start us, avg end us)} relative to the first
        stamp of each step row -- the in-step schedule of every launch (all
        streams), over the rows where that launch was stamped"""
        st = self.stamps.cpu().view(self.rows, len(NAMES), PER_ID, 2).to(torch.int64)
        valid = (st > 0).view(self.rows, -1)
        rows = valid.any(1)
        st, valid = st[rows], valid[rows]
        if st.shape[0] == 0:
            return {}
        big = torch.iinfo(torch.int64).max
        t0 = torch.where(valid, st.view(st.shape[0], -1), torch.full_like(st.view(st.shape[0], -1), big)).min(1).values
        out = {}
        for k, n in enumerate(NAMES):
            for i in range(PER_ID):
                a, b = st[:, k, i, 0], st[:, k, i, 1]
                ok = (a > 0) & (b >= a)
                if ok.any():
                    sa = ((a - t0)[ok].double() * self.tick_ns * 1e-3).mean().item()
                    sb = ((b - t0)[ok].double() * self.tick_ns * 1e-3).mean().item()
                    out[f"{n}#{i}"] = (round(sa, 1), round(sb, 1))
        return dict(sorted(out.items(), key=lambda kv: kv[1][0]))

    def steps(self):
        st = self.stamps.view(self.rows, -1)
        return int((st > 0).any(1).sum())

    def summary(self):
        """{kernel: (avg ms per launch, launches per step)} over the steps recorded"""
        n = max(1, self.steps())
        return {k: (sum(v) / len(v), len(v) / n) for k, v in self.read().items()}


# include/ngp_amd.h NGP_P_* order
PROBES = ["march", "first_chunk", "field_encode_mlp", "composite_loss", "mlp_bwd", "hash_bwd_coarse", "hash_count",
          "hash_write", "hash_accum", "adam", "segments", "rays_nonempty", "counters_inc", "hash_plan", "adam_residual",
          "march_compact", "sample_batch", "pre_encode"]


class ProbeTimer:
    """Execution spans of the probed kernels (ngp_probe_set: lane 0 of each
    wave of a probed kernel stores its start and end time into its own slot
    of a row chosen by the device step counter; the span = min start .. max
    end).  No graph node is added, so the graphs already captured replay
    unchanged with the probes on: the spans are those of the product step,
    comparable launch for launch with a rocprofv3 kernel trace of the same
    replays.  rows: steps kept (row = step % rows: a window longer than rows
    keeps its last `rows` steps).  Usage: arm(); run steps; disarm();
    summary(skip_rows=...)."""

    WAVES = 65536  # NGP_PROBE_WAVES

    def __init__(self, step_counter, rows=32, device="cuda"):
        assert _lib().ngp_probe_count() == len(PROBES)
        self.step = step_counter
        self.rows = rows
        self.buf = torch.zeros(rows, len(PROBES), self.WAVES, 2, dtype=torch.int64, device=device)
        self.tick_ns = _lib().ngp_timing_tick_ns()

    def reset(self):
        self.buf.zero_()

    def arm(self):
        torch.cuda.synchronize()
        self.reset()
        vren._ok(_lib().ngp_probe_set(self.buf.data_ptr(), self.step.data_ptr(), self.rows), "probe_set")

    def disarm(self):
        torch.cuda.synchronize()
        vren._ok(_lib().ngp_probe_set(None, None, 0), "probe_set")

    def spans(self, skip_rows=()):
        """{probe: [(row, ms), ...]} for every row where the probe ran, rows in skip_rows excluded"""
        b = self.buf
        big = torch.iinfo(torch.int64).max
        st = torch.where(b[..., 0] > 0, b[..., 0], torch.full_like(b[..., 0], big)).min(-1).values.cpu()
        en = b[..., 1].max(-1).values.cpu()
        ok = (en > 0) & (st < big) & (en >= st)
        ms = (en - st).double() * self.tick_ns * 1e-6
        skip = set(skip_rows)
        out = {}
        for k, n in enumerate(PROBES):
            rows = [r for r in torch.nonzero(ok[:, k]).flatten().tolist() if r not in skip]
            if rows:
                out[n] = [(r, float(ms[r, k])) for r in rows]
        return out

    def summary(self, skip_rows=()):
        """{probe: (avg ms per launch, launches counted)}"""
        return {k: (sum(m for _, m in v) / len(v), len(v)) for k, v in self.spans(skip_rows).items()}

    def step_gaps(self, step0, n_steps, skip_steps=(), first="first_chunk", last="counters_inc"):
        """[(step, us)]: from the end of step s's `last` kernel to the start of
        step s + 1's `first` (the step boundary: inside a two-step graph, or
        between two graph replays), for the consecutive steps s, s + 1 of the
        window [step0, step0 + n_steps) (n_steps <= rows: rows are step % rows,
        so only pairs inside the window are taken -- the row after the
        window's last step holds its FIRST step) where neither is in
        skip_steps (steps with an occupancy update launch extra kernels)"""
        b = self.buf
        big = torch.iinfo(torch.int64).max
        st = torch.where(b[..., 0] > 0, b[..., 0], torch.full_like(b[..., 0], big)).min(-1).values.cpu()
        en = b[..., 1].max(-1).values.cpu()
        f, l = PROBES.index(first), PROBES.index(last)
        skip = set(skip_steps)
        out = []
        for s in range(step0, step0 + min(n_steps, self.rows) - 1):
            if s in skip or s + 1 in skip:
                continue
            r, r1 = s % self.rows, (s + 1) % self.rows
            if en[r, l] > 0 and st[r1, f] < big:
                out.append((s, round(float(st[r1, f] - en[r, l]) * self.tick_ns * 1e-3, 1)))
        return out

    def step_periods(self, step0, n_steps, first="first_chunk"):
        """[(step, us)]: from the start of step s's `first` kernel to the start
        of step s + 1's, for the consecutive steps of the window [step0, step0 +
        n_steps) (as step_gaps) -- a step's whole period, including the
        occupancy update and the march that follow it when step s + 1 opens
        with one"""
        b = self.buf
        big = torch.iinfo(torch.int64).max
        st = torch.where(b[..., 0] > 0, b[..., 0], torch.full_like(b[..., 0], big)).min(-1).values.cpu()
        f = PROBES.index(first)
        out = []
        for s in range(step0, step0 + min(n_steps, self.rows) - 1):
            r, r1 = s % self.rows, (s + 1) % self.rows
            if st[r, f] < big and st[r1, f] < big:
                out.append((s, round(float(st[r1, f] - st[r, f]) * self.tick_ns * 1e-3, 1)))
        return out

    def timeline(self, skip_rows=(), origin="first_chunk"):
        """{probe: (avg start us, avg end us)} relative to the start of `origin`
        in the same step row: the step's schedule as the kernels ran (no
        stamp kernels in the graph), over the rows where both ran"""
        b = self.buf
        big = torch.iinfo(torch.int64).max
        st = torch.where(b[..., 0] > 0, b[..., 0], torch.full_like(b[..., 0], big)).min(-1).values.cpu()
        en = b[..., 1].max(-1).values.cpu()
        o = PROBES.index(origin)
        skip = set(skip_rows)
        out = {}
        for k, n in enumerate(PROBES):
            rows = [r for r in range(self.rows) if r not in skip and en[r, k] > 0 and st[r, k] < big
                    and en[r, o] > 0 and st[r, o] < big]
            if rows:
                s0 = sum(float(st[r, k] - st[r, o]) for r in rows) / len(rows) * self.tick_ns * 1e-3
                e0 = sum(float(en[r, k] - st[r, o]) for r in rows) / len(rows) * self.tick_ns * 1e-3
                out[n] = (round(s0, 1), round(e0, 1))
        return dict(sorted(out.items(), key=lambda kv: kv[1][0]))
