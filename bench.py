#!/usr/bin/env python
"""xRT benchmark: large-v3, beam 5, fp16, synthetic audio, 1..8 MI355X (one process per GPU).

A "step" is one ``transcribe()`` of a file through the multi-GPU path of SURVEY.md
§8(e) (whisper/distributed.py): every rank computes the log-mel of its block of 30 s
clips from the audio resident in its HBM, the log-mel maximum is all-reduced (MAX,
RCCL), each rank decodes its clips (batched schedule: all its windows through the
encoder and the hipGraph decoder step together), and the segment records are gathered
on rank 0.  condition_on_previous_text = False, temperature 0.

Default (weak scaling, BASELINE config 3 at N = 1): the file holds ``--seconds``
(600) of audio per rank.  ``--sharded-file 1`` (config 4): one file of ``--seconds``
(e.g. 3600) in total, whatever the rank count (strong scaling).  With more than one
rank, rank 0 re-transcribes the whole file unsharded after the timed region and
reports whether the merged segments equal it (``verify``).

value = (audio seconds of the whole file x steps) / (max over ranks of the timed
wall time) = whole-job xRT.  rank 0 prints one JSON line.

Launch: under torch.distributed.run (WORLD_SIZE set) every process is one rank.
Without it, ``--gpus N`` > 1 starts the N ranks itself (``launch_ranks``): N child
processes of this script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
spawned before this process touches the GPU; the parent waits for all of them and
exits non-zero if any rank fails.  Every rank checks world == --gpus.
"""

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "whisper.coreml_amd"))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
MFMA_F16_PEAK_TFS = 2500.0  # dense fp16/bf16 MFMA, spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", default="large-v3")
    p.add_argument("--seconds", type=float, default=600.0,
                   help="audio seconds per GPU (weak scaling); with --sharded-file, of the whole file")
    p.add_argument("--sharded-file", type=int, default=0,
                   help="config 4: one file of --seconds sharded over the ranks (strong scaling)")
    p.add_argument("--verify", type=int, default=-1,
                   help="rank 0 compares the merged segments with an unsharded run (default: when > 1 rank)")
    p.add_argument("--latency", type=int, default=1,
                   help="also time single-window decoding (1 window x beam: the per-token p50 of §8(d))")
    p.add_argument("--beam", type=int, default=5)
    p.add_argument("--dtype", default="fp16")
    p.add_argument("--max-windows", type=int, default=20)
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--cpu-steps", type=int, default=48,
                   help="CPU baseline: beam decoder steps of its window, the step part scaled to the window's 224 "
                        "(a bounded sample: ~20-25 s of CPU work on 16 cores; 0 = the whole 224-step window, ~90 s)")
    p.add_argument("--dump", default="", help="write the last step's segments (tokens, avg_logprob) as JSON")
    p.add_argument("--word-timestamps", type=int, default=0,
                   help="config 5: transcribe(word_timestamps=True) (alignment + DTW on the GPU per window)")
    p.add_argument("--backend", default="nccl", help="torch.distributed backend of the ranks (nccl = RCCL)")
    p.add_argument("--launch-check", type=int, default=0,
                   help="only bring the ranks up, all-gather (rank, world) and print it from rank 0 (no GPU work)")
    p.add_argument("--launch-check-fail-rank", type=int, default=-1,
                   help="(launcher test) with --launch-check: this rank exits 3 after init while the others wait "
                        "in a collective")
    p.add_argument("--dist-timeout", type=float, default=900.0,
                   help="seconds before a torch.distributed collective gives up")
    p.add_argument("--balance", default="clips", choices=("clips", "tokens"),
                   help="clips per rank: contiguous blocks (clips: equal clip counts, fixed work) or every N-th clip "
                        "(tokens: natural decoding, where EOTs and speech density make windows unequal)")
    return p.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, poll_s=0.2, grace_s=10.0):
    """--gpus N without an external launcher: run this script as N rank processes.

    Called before anything in this process imports torch.cuda or the HIP library
    (no exec: the children are new processes, this one only waits).  The children are
    polled together: the first one to exit non-zero ends the run — its siblings (which
    may be blocked in a collective waiting for it) get SIGTERM, then SIGKILL after
    ``grace_s`` — and its code is returned.  0 when every rank exited 0."""
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    failed = None  # (rank, code) of the first rank that failed
    while failed is None and any(p.poll() is None for p in procs):
        for r, p in enumerate(procs):
            c = p.poll()
            if c is not None and c != 0:
                failed = (r, c)
                break
        else:
            time.sleep(poll_s)
    if failed is None:
        failed = next(((r, p.returncode) for r, p in enumerate(procs) if p.returncode != 0), None)
    if failed is None:
        return 0
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.monotonic() + grace_s
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    print(f"bench.py: rank {failed[0]} failed with exit code {failed[1]}; "
          f"rank(s) failed: {[(r, p.returncode) for r, p in enumerate(procs) if p.returncode != 0]}",
          file=sys.stderr, flush=True)
    return failed[1] if failed[1] > 0 else 1


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}")
    pg = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            import torch
            torch.cuda.set_device(local)
        from datetime import timedelta
        # bounded collectives: a rank that never arrives ends the run with an error
        # instead of a hang (the launcher above also ends the survivors of a dead rank)
        dist.init_process_group(args.backend, timeout=timedelta(seconds=args.dist_timeout))
        assert dist.get_world_size() == args.gpus
        pg = dist
    return world, rank, local, pg


def parallelism_label(world, file_seconds, balance):
    """config.parallelism: what the run's ranks exchange (nothing at world 1)."""
    if world == 1:
        return (f"one {file_seconds:.0f} s file on 1 GPU by 30 s clips (whisper/distributed.py, world 1: "
                f"no collective runs)")
    return (f"one {file_seconds:.0f} s file sharded over {world} GPUs by 30 s clips "
            f"({'contiguous blocks' if balance == 'clips' else 'every ' + str(world) + '-th clip'}, "
            f"whisper/distributed.py): RCCL all-reduce(max) of the log-mel maximum + gather of the segment records")


def per_rank_report(pg, rec):
    """Every rank's record (wall time, windows, tokens, time in the two collectives) on
    every rank, in rank order: the N > 1 line shows why a scaling curve bends."""
    if pg is None:
        return [rec]
    out = [None] * pg.get_world_size()
    pg.all_gather_object(out, rec)
    return out


def launch_check(args):
    """--launch-check 1: the ranks came up; rank 0 prints every rank's (rank, world) and
    the per-rank record the bench line carries (no GPU work: times are zero)."""
    world, rank, _, pg = dist_setup(args)
    seen = [(rank, world)]
    if pg is not None and rank == args.launch_check_fail_rank:
        os._exit(3)  # dies after init; the other ranks block in the all-gather below
    if pg is not None:
        seen = [None] * world
        pg.all_gather_object(seen, (rank, pg.get_world_size()))
    per_rank = per_rank_report(pg, dict(rank=rank, wall_s=0.0, windows=0, tokens=0, global_max_s=0.0, gather_s=0.0))
    if rank == 0:
        line = {"launch_check": True, "n_gpus": world, "ranks": seen,
                "parallelism": parallelism_label(world, 600.0 * world, args.balance)}
        if world > 1:
            line["per_rank"] = per_rank
        print(json.dumps(line), flush=True)
    if pg is not None:
        pg.destroy_process_group()


def allreduce_max(pg, x: float) -> float:
    if pg is None:
        return x
    from whisper import distributed as D
    return D.global_max(x)  # RCCL on a device tensor under nccl, a CPU tensor under gloo


def barrier(pg):
    if pg is not None:
        pg.barrier()


def decoder_step_bytes(dims, n_windows, beams, mean_ctx, elem=2):
    """Algorithmic HBM bytes of one decoder step: decoder weights
    (L*14 n^2 + V n params, read once per step for the whole batch), the cross-KV of
    every window (2 * 1500 * n * L), the self-KV of every beam row (2 * t * n * L)."""
    n, L, V = dims["n_text_state"], dims["n_text_layer"], dims["n_vocab"]
    weights = (L * 14 * n * n + V * n) * elem
    cross = n_windows * 2 * 1500 * n * L * elem
    selfkv = n_windows * beams * 2 * mean_ctx * n * L * elem
    return weights + cross + selfkv


def projection_bytes_per_launch(dims, rows, p1, elem=2, fused_q=False):
    """Algorithmic bytes of one decoder-step projection launch, averaged over the ones a
    decoder layer runs: qkv n->3n, out n->n, cross-q n->n, cross-out n->n, fc1 n->4n,
    fc2 4n->n — without the cross-q when the step projects it inside the cross-attention
    (`fused_q`, round 6: five per layer).  Split-K k_proj: weights N*K + activations
    rows*K (fp16) + the result rows*N (fp16 slabs in fp16 contexts, counted at 4 B: the
    algorithmic output of the projection, not its slab format).  k_proj1 (`p1`): weights
    N*K; the LayerNorm'd projections read the fp32 residual rows*K*4 + gamma/beta and write
    rows*N fp16; the residual ones read rows*K fp16 and read + write the fp32 residual
    rows*N*4*2."""
    n = dims["n_text_state"]
    if p1:
        ln = [(3 * n, n), (4 * n, n)] + ([] if fused_q else [(n, n)])
        res = [(n, n), (n, n), (n, 4 * n)]
        tot = sum(N * K * elem + rows * K * 4 + 2 * K * 4 + rows * N * elem for N, K in ln)
        tot += sum(N * K * elem + rows * K * elem + rows * N * 8 for N, K in res)
        return tot // (len(ln) + len(res))
    shapes = [(3 * n, n), (n, n), (n, n), (4 * n, n), (n, 4 * n)] + ([] if fused_q else [(n, n)])
    tot = sum(N * K * elem + rows * K * elem + rows * N * 4 for N, K in shapes)
    return tot // len(shapes)


def cross_attn_bytes_per_launch(dims, n_windows, rows, elem=2, fused_q=False):
    """One layer's cross-attention: K and V of every window (2*1500*n) + q in / out; with
    the query projected in the kernel (round 6) + the query weights n*n (the rows in are
    the LayerNorm'd rows instead of q: the same rows*n)."""
    n = dims["n_text_state"]
    return n_windows * 2 * 1500 * n * elem + 2 * rows * n * elem + (n * n * elem if fused_q else 0)


def load_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC pass
    (profiles/<round>/traffic.json, written by profiles/pmc_traffic.py: FETCH_SIZE x2
    + WRITE_SIZE per the gfx950 correction of MI355X_MICROARCH.md), or None."""
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        path = os.path.join(REPO, "profiles", rnd, "traffic.json")
        try:
            with open(path) as f:
                return json.load(f)[kernel]["hbm_bytes_per_launch"]
        except (OSError, KeyError, ValueError):
            continue
    return None


def encoder_flops(dims):
    n, L, T = dims["n_audio_state"], dims["n_audio_layer"], 1500
    conv = 2 * 3000 * dims["n_mels"] * 3 * n + 2 * 1500 * n * 3 * n
    block = 2 * T * n * (3 * n) + 2 * 2 * T * T * n + 2 * T * n * n + 2 * 2 * T * n * 4 * n
    return conv + L * block


def cpu_topology():
    """Threads for the CPU baseline (the physical cores of one socket).

    The physical cores of the socket holding most of this process's allowed CPUs
    (os.sched_getaffinity + sysfs topology), capped by the CPU share the process is
    given: the cgroup cpu.max quota, else OMP_NUM_THREADS when the environment sets it
    (the GPU pool gives each one-GPU job a 16-CPU share and exports 16)."""
    allowed = sorted(os.sched_getaffinity(0))
    sockets = {}
    for c in allowed:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            with open(base + "physical_package_id") as f:
                pkg = int(f.read())
            with open(base + "core_id") as f:
                core = int(f.read())
        except (OSError, ValueError):
            pkg, core = 0, c
        sockets.setdefault(pkg, set()).add(core)
    socket_cores = max((len(v) for v in sockets.values()), default=len(allowed))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() else None
    share, why = None, "one socket's physical cores"
    if quota is not None:
        share, why = quota, f"capped by the cgroup CPU quota ({quota} CPUs)"
    elif omp is not None:
        share, why = omp, f"capped by the job's CPU share (OMP_NUM_THREADS={omp})"
    threads = min(socket_cores, share) if share else socket_cores
    if share and share >= socket_cores:
        why = "one socket's physical cores"
    return dict(threads=threads, socket_physical_cores=socket_cores, sockets=len(sockets), allowed_cpus=len(allowed),
                cgroup_cpus=quota, omp_num_threads=omp, why=why)


def cpu_baseline(model_name, sd, audio, beams, n_steps):
    """The oracle (CPU fp32 restatement, oracle/ref_whisper.py) decoding one 30 s window
    exactly as the reference's DecodingTask does (encoder, first pass, then every
    beam-search step with its filters, top-k candidate merge and KV reorder) with
    fixed work (EOT suppressed: 224 steps).  n_steps > 0 stops after that many
    steps and scales the step part to 224 (a bounded sample)."""
    import torch
    from oracle import ref_whisper as R
    from whisper import synthetic as S
    topo = cpu_topology()
    torch.set_num_threads(topo["threads"])
    threads = torch.get_num_threads()
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next(line.split(":", 1)[1].strip() for line in f if line.startswith("model name"))
    except (OSError, StopIteration):
        pass
    dims = S.MODEL_DIMS[model_name]
    m = R.OracleWhisper(dims, sd)
    st = R.SpecialTokens.for_model(dims)
    mel = R.pad_or_trim(R.log_mel_spectrogram(audio[:480000], dims["n_mels"], padding=R.N_SAMPLES)[:, :3000])
    t0 = time.time()
    xa = m.encode(mel)
    t_enc = time.time() - t0
    opts = R.Options(beam_size=beams, suppress_tokens=f"-1,{st.eot}", sample_len=n_steps or None)
    t0 = time.time()
    res = R.decode(m, mel, opts, st, xa=xa)
    t_dec = time.time() - t0
    steps = n_steps or 224
    per_window = t_enc + t_dec * (224 / steps)
    kind = "the whole window" if not n_steps else f"{steps} steps scaled to 224"
    return dict(value=round(30.0 / per_window, 4), unit="xRT (audio-s/s)", cores=threads, cpu_model=cpu_model,
                kind="port", topology=topo,
                sample=f"1 window (30 s) of {model_name}, beam {beams}, {kind}: encoder {t_enc:.1f} s + decode "
                       f"{t_dec:.1f} s ({len(res.tokens)} tokens; oracle/ref_whisper.py decode with the reference's "
                       f"beam search, torch CPU fp32, {threads} threads of {cpu_model})")


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.launch_check:
        return launch_check(args)
    world, rank, local, pg = dist_setup(args)
    import whisper
    from whisper import distributed as D
    from whisper import synthetic as S

    dims = S.MODEL_DIMS[args.model]
    from whisper.backend_hip import max_windows_limit
    lim = max_windows_limit(dims, args.dtype, args.beam)
    if args.max_windows > lim:
        print(f"bench.py: --max-windows {args.max_windows} exceeds what one context holds at beam {args.beam} in "
              f"{args.dtype} (self-KV cache per layer < 2 GiB): using {lim}", file=sys.stderr, flush=True)
        args.max_windows = lim
    sd = S.synthetic_state_dict(dims, 0)
    model = whisper.Whisper(whisper.ModelDimensions(**dims), args.model, device=local, dtype=args.dtype,
                            max_windows=args.max_windows, max_group=args.beam)
    model.load_state_dict(sd)
    if args.model in whisper._ALIGNMENT_HEADS:  # as load_model does (reference __init__.py:176-177)
        model.set_alignment_heads(whisper._ALIGNMENT_HEADS[args.model])
    if not (rank == 0 and world == 1 and args.cpu_baseline):
        del sd
        sd = None
    if args.word_timestamps and world > 1:
        raise SystemExit("--word-timestamps is a single-GPU workload (config 5): sharding refuses it")
    file_seconds = args.seconds if args.sharded_file else args.seconds * world
    n_clips = int(round(file_seconds / 30.0))
    # one seeded file, resident in every rank's HBM before the timed region
    audio = S.synthetic_audio(file_seconds, seed=1000)
    dev_audio = model.ctx.audio_upload(audio)
    decode_kw = dict(temperature=0.0, beam_size=args.beam, language="en")

    # per-rank accounting of the timed steps (the N > 1 line's per_rank records)
    acct = dict(global_max_s=0.0, gather_s=0.0, windows=0, tokens=0)

    def one_step():
        if args.word_timestamps:
            # config 5 on one GPU: the same clip grid, words aligned on the GPU per window
            clip_ts = ",".join(f"{30 * i},{30 * (i + 1)}" for i in range(n_clips))
            return whisper.transcribe(model, dev_audio, condition_on_previous_text=False, clip_timestamps=clip_ts,
                                      schedule="batched", word_timestamps=True, **decode_kw)["segments"]
        st = D.prepare_shard(model, dev_audio, rank, world, args.balance)
        t = time.perf_counter()
        g = allreduce_max(pg, st.local_max)
        acct["global_max_s"] += time.perf_counter() - t
        segs = D.run_shard(model, st, g, balance=args.balance, **decode_kw)
        acct["windows"] += len(st.clips)
        acct["tokens"] += sum(len(s["tokens"]) for s in segs)
        if pg is None:
            return D.merge_segments([segs])
        t = time.perf_counter()
        merged = D.gather_segments(segs)  # rank 0: the merged file; others: None
        acct["gather_s"] += time.perf_counter() - t
        return merged

    for _ in range(args.warmup):
        one_step()
    acct.update(global_max_s=0.0, gather_s=0.0, windows=0, tokens=0)
    barrier(pg)
    model.ctx.sync()
    st0 = model.ctx.stats()
    model.ctx.token_ms(reset=True)
    t0 = time.perf_counter()
    results = []
    for _ in range(args.steps):
        results.append(one_step())
    model.ctx.sync()
    barrier(pg)
    elapsed = time.perf_counter() - t0
    st1 = model.ctx.stats()
    elapsed_max = allreduce_max(pg, elapsed)
    per_rank = per_rank_report(pg, dict(rank=rank, wall_s=round(elapsed, 4), windows=acct["windows"],
                                        tokens=acct["tokens"], global_max_s=round(acct["global_max_s"], 5),
                                        gather_s=round(acct["gather_s"], 5)))
    merged = results[-1]

    if args.dump and rank == 0:
        with open(args.dump, "w") as f:
            json.dump([{k: s[k] for k in ("seek", "tokens", "avg_logprob", "no_speech_prob")} for s in merged], f)

    verify = None
    if (args.verify if args.verify >= 0 else world > 1) and rank == 0:
        # the whole file on this GPU alone, same options, unsharded: the merged records must equal it
        clip_ts = ",".join(f"{30 * i},{30 * (i + 1)}" for i in range(n_clips))
        ref = whisper.transcribe(model, audio, condition_on_previous_text=False, clip_timestamps=clip_ts,
                                 schedule="batched", **decode_kw)["segments"]
        same = [a["tokens"] == b["tokens"] and a["seek"] == b["seek"] for a, b in zip(merged, ref)]
        verify = {"segments": len(merged), "unsharded_segments": len(ref),
                  "equal": len(merged) == len(ref) and all(same),
                  "segments_equal_frac": round(sum(same) / max(len(ref), 1), 4)}

    seg_tokens = sum(len(s["tokens"]) for s in merged) if merged is not None else 0
    steps_done = st1["steps"] - st0["steps"]
    steps_ms = st1["steps_ms"] - st0["steps_ms"]
    enc_ms = st1["encode_ms"] - st0["encode_ms"]
    enc_windows = st1["encode_windows"] - st0["encode_windows"]
    ms_per_token = steps_ms / max(steps_done, 1)
    per_rank_windows = -(-n_clips // world)
    n_win = min(args.max_windows, per_rank_windows)
    # p50 per-token decode ms: median over the timed region's decode_steps chunks
    tok = model.ctx.token_ms()
    p50_token_ms = float(np.median(tok)) if len(tok) else ms_per_token

    # overall roofline: the encoder's flops at the dense fp16 MFMA peak plus
    # every decoder step's bytes at the HBM peak, over the measured wall time
    mean_ctx = 3 + 112  # mid-window self-KV length for the byte count
    ideal_s = (encoder_flops(dims) * enc_windows / (MFMA_F16_PEAK_TFS * 1e12)
               + steps_done * decoder_step_bytes(dims, n_win, args.beam, mean_ctx) / (HBM_PEAK_GBS * 1e9))
    overall = {"ideal_ms_per_step": round(ideal_s * 1e3 / args.steps, 2),
               "frac": round(ideal_s / elapsed, 4),
               "model": "encoder flops / 2.5 PFLOP/s + decoder step bytes (weights + cross-KV + self-KV at "
                        "mean context 115) / 8 TB/s, rank-local"}

    # roofline of the dominant kernel (k_proj: the split-K projections of the decoder
    # step), timed live with HIP events on the context's stream over launches at the
    # bench batch (all layers, so weights stream from HBM)
    model.ctx.encode([3000 * i for i in range(n_win)], [3000] * n_win)
    from whisper.decoding import DecodingTask
    task = DecodingTask(model, whisper.DecodingOptions(language="en", beam_size=args.beam))
    model.ctx.decode_begin(task.wh_opts(), [task.initial_tokens] * n_win, [task.sot_index] * n_win)
    rows = n_win * args.beam
    # in-step: every k_proj of 6 eager steps bracketed by HIP events on the context
    # stream, each behind its real producer kernel (what rocprof sees in the step);
    # back-to-back: the same launches queued without their producers (time_stage 2)
    model.ctx.time_stage(7, 2)  # warm-up (without it the same tree read 7.0-8.1 us run to run)
    gemv_ms = model.ctx.time_stage(7, 6)
    gemv_b2b_ms = model.ctx.time_stage(2, 3)
    kern = model.ctx.step_kernels(n_win, args.beam)  # what the library runs for this batch
    p1 = kern["proj"] == "k_proj1"
    fused_q = "<qproj" in kern["xattn"]  # the cross-q projected inside the cross-attention (round 6)
    gemv_bytes = projection_bytes_per_launch(dims, rows, p1, fused_q=fused_q)
    xattn_ms = model.ctx.time_stage(3, 3)
    xattn_bytes = cross_attn_bytes_per_launch(dims, n_win, rows, fused_q=fused_q)
    step_ms = model.ctx.time_stage(0, 20)
    step_bytes = decoder_step_bytes(dims, n_win, args.beam, mean_ctx)

    # single-window decoding (§8(d)'s p50: one _main_loop iteration at B = beam): one
    # window, the whole 224-step fixed-work decode through decode_steps, per-token wall
    # time of each 8-step chunk (graph launches + the host's done poll)
    latency = None
    if args.latency:
        model.ctx.encode([0], [3000])
        t1 = DecodingTask(model, whisper.DecodingOptions(language="en", beam_size=args.beam,
                                                         suppress_tokens=f"-1,{task.tokenizer.eot}"))
        model.ctx.decode_begin(t1.wh_opts(), [t1.initial_tokens], [t1.sot_index])
        model.ctx.token_ms(reset=True)
        model.ctx.decode_steps(t1.sample_len)
        tk1 = model.ctx.token_ms(reset=True)
        # the step graph alone, on a live window (after decode_steps the window is done and
        # the selection / merge would return early): begin the batch again, then 20 replays
        model.ctx.decode_begin(t1.wh_opts(), [t1.initial_tokens], [t1.sot_index])
        step1 = model.ctx.time_stage(0, 20)
        latency = {"p50_token_ms_1window": round(float(np.median(tk1)), 4), "step_graph_ms_1window": round(step1, 4),
                   "step_bytes_1window": decoder_step_bytes(dims, 1, args.beam, mean_ctx),
                   "roofline_frac_1window": round(decoder_step_bytes(dims, 1, args.beam, mean_ctx) /
                                                  (step1 * 1e-3) / (HBM_PEAK_GBS * 1e9), 4)}

    def gbs(b, ms):
        return b / (ms * 1e-3) / 1e9

    # the committed PMC pass (profiles/pmc_traffic.py) ran large-v3 at 20 windows (k_proj,
    # k_xattn_seg) and at one window (k_proj1): other shapes report no traffic
    lv3 = args.model == "large-v3"
    traffic = load_traffic(kern["proj"]) if lv3 and (p1 or n_win == 20) else None
    xattn_traffic = load_traffic(kern["xattn"].split("<")[0]) if lv3 and n_win == 20 else None
    parallel = parallelism_label(world, file_seconds, args.balance)
    out = {
        "metric": "xRT (audio-s/s) large-v3 beam=5 @1/2/4/8 GPU; p50 per-token decode ms",
        "value": round(file_seconds * args.steps / elapsed_max, 3),
        "unit": "audio-s/s",
        "n_gpus": pg.get_world_size() if pg is not None else world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max * 1e3 / args.steps, 2),
        "higher_is_better": True,
        "scaling": "strong" if args.sharded_file else "weak",
        "vs_baseline": None,
        "dtype": "fp16" if args.dtype == "fp16" else "f32",
        "data": "synthetic: seeded N(0,0.1^2)+440 Hz audio, seeded random-init weights at real dims",
        "config": {"workload": f"{args.model} beam={args.beam} transcribe() of one {file_seconds:.0f} s file, "
                               f"30 s clip grid, condition_on_previous_text=False, temperature=0"
                               + (", word_timestamps=True" if args.word_timestamps else ""),
                   "model": args.model, "global_batch": n_clips, "seq_len": 448, "parallelism": parallel},
        # §8(d): one _main_loop iteration at B = beam for a single window; the batch
        # figures are the same per-token wall time with every window of the rank decoding
        "p50_token_ms": latency["p50_token_ms_1window"] if latency else round(p50_token_ms, 4),
        "p50_token_ms_batch": round(p50_token_ms, 4),
        "mean_token_ms_batch": round(ms_per_token, 4),
        "tokens_per_window": round(seg_tokens / max(1, n_clips), 1) if rank == 0 else None,
        "encoder_ms_per_window": round(enc_ms / max(enc_windows, 1), 3),
        "encoder_tflops": round(encoder_flops(dims) * enc_windows / (enc_ms * 1e-3) / 1e12, 1) if enc_ms else None,
        "roofline": {"bound": "hbm", "kernel": (f"k_proj1 whole-K projection, fused LayerNorm / epilogue ({rows} rows"
                                                if p1 else f"k_proj split-K projection ({rows} rows")
                                               + f", avg of the {'five' if fused_q else 'six'} per decoder layer)",
                     "achieved": round(gbs(gemv_bytes, gemv_ms), 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(gbs(gemv_bytes, gemv_ms) / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "bytes_per_launch": gemv_bytes, "ms_per_launch": round(gemv_ms, 5),
                     "timing": "HIP events around each launch inside eager decoder steps",
                     "launches_per_layer": 5 if fused_q else 6,
                     "ms_per_launch_back_to_back": round(gemv_b2b_ms, 5),
                     "back_to_back_note": "time_stage 2: the layer's projections queued without their "
                                          "producers; on the k_proj1 path the non-deferred fc2 and the plain QKV "
                                          "LayerNorm prologue (the step itself defers fc2's residual)"},
        "roofline_overall": overall,
        "roofline_cross_attn": {"bound": "hbm", "kernel": f"{kern['xattn']} ({n_win} windows x {args.beam} beams)",
                                "achieved": round(gbs(xattn_bytes, xattn_ms), 1), "peak": HBM_PEAK_GBS,
                                "frac": round(gbs(xattn_bytes, xattn_ms) / HBM_PEAK_GBS, 4),
                                "traffic": xattn_traffic,
                                "bytes_per_launch": xattn_bytes, "ms_per_launch": round(xattn_ms, 5)},
        "roofline_step": {"bound": "hbm", "kernel": f"decoder step hipGraph ({n_win} windows x {args.beam} beams)",
                          "achieved": round(gbs(step_bytes, step_ms), 1), "peak": HBM_PEAK_GBS,
                          "frac": round(gbs(step_bytes, step_ms) / HBM_PEAK_GBS, 4),
                          "bytes_per_launch": step_bytes, "ms_per_launch": round(step_ms, 4)},
    }
    if latency:
        out["latency_1window"] = latency
    if world > 1:
        # per rank over the timed steps: wall time, windows and segment tokens decoded, and
        # the seconds spent in the two collectives (all-reduce MAX, segment gather)
        out["per_rank"] = per_rank
        out["balance"] = args.balance
    if verify is not None:
        out["verify"] = verify
    if rank == 0 and world == 1 and args.cpu_baseline and sd is not None:
        try:
            out["cpu_baseline"] = cpu_baseline(args.model, sd, audio, args.beam, args.cpu_steps)
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
