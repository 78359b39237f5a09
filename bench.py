#!/usr/bin/env python3
"""bench.py — BASELINE metric of the MI355X-native MioTTS path.

Metric (BASELINE.json): realtime factor (audio s / wall s) + stage ms llm/codec/istft on
MioTTS-1.7B Q4_K_M (configs[2]): one "step" = one whole utterance of the reference
pipeline (test-to-speech.cpp:94-246): chat-template prompt -> prefill -> 700 sampled
speech tokens (temp 0.8, on-device sampler, speech ids only so synthetic weights yield
exactly 700 codes: flagged harness deviation) -> MioCodec decode -> iSTFT ->
PCM left in HBM (`value`; the PCIe-inclusive rate with the PCM copied to host memory is
reported beside it as `value_pcie_inclusive`). Weights are synthetic (no checkpoints
offline) with the published shapes; "data": "synthetic".

Multi-GPU (`--gpus N`): one process per GPU. Under torchrun (WORLD_SIZE set) this process
is one rank; otherwise, for N > 1, it starts N fresh child processes of itself (RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_* set) BEFORE anything touches the GPU and exits with
their status. Each rank synthesizes its own utterances (independent: no collective on the
data path, "scaling": "weak"); a gloo barrier brackets the timed region and the max
elapsed over ranks is used. `--utts-per-gpu B` makes every step B utterances decoded
together by the batched engine on each rank (BASELINE configs[3], C4: `--preset 4
--utts-per-gpu 8 --gpus 8` = 64 utterances of the 2.6B Q8_0 model over 8 GPUs).

roofline: the decode-step kernel with the largest in-graph time per token (step timeline,
mio_hip_llm_timeline, after the timed region at decode position ~400 = the utterance's mean
position and the PMC run's): achieved = its algorithmic bytes per launch (GGUF bytes of the matrices it streams +
activations; attention: the F16 K/V rows of positions <= pos + q/k/v in + partial records
out, mio_hip_llm_time_kernel) / its mean launch duration from HIP events around a replayed
graph of 40 back-to-back launches on the runner's stream (the fused launches: each behind a
memset of their hand-off counters, minus a replayed graph of the memsets alone; GPU-paced,
within 4 % of the eager rocprof means, profiles/r06/time_kernel_modes.txt); peak = 8 TB/s HBM3E. `frac_in_graph` = the
same bytes over the in-graph span (first workgroup start -> last workgroup end,
s_memrealtime; the timeline replays the diagnostic kernel instantiations). traffic = the same kernel's HBM bytes per launch
from rocprofv3 PMC (FETCH_SIZE x 2 on gfx950 + WRITE_SIZE, profiles/pmc_traffic.json,
tools/pmc_traffic.py). step_* = all bytes of one decode step over the step's graph wall.
cpu_baseline: the C oracle (oracle/, "port") on rank 0 at N=1 only, timed on a bounded
sample (decode steps at positions spread over 0..700 + codec/iSTFT of a few codes) and
extrapolated to one utterance, at the box's thread share and at 4 threads.
baseline_configs (N=1, after everything else; --no-configs skips): the other BASELINE configs,
each in a child process with its own timed region at short K — C2 (0.1B Q8_0), C4 per GPU on
the 2.6B Q8_0 stand-in and on the LFM2-2.6B shape (8 utterances decoded together), and C5 (the
miotts-stream-benchmark CLI's own clock); never part of `value`.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
ROOF_POS = 400  # decode position of the roofline timeline / kernel timings (and of the PMC run)
KERNEL_NAMES = {0: "k_attn_in", 1: "k_attention", 2: "k_attn_out", 3: "k_ffn_in", 4: "k_ffn_down",
                6: "k_lm_head", 8: "k_conv_in", 9: "k_conv_out", 10: "k_att_o", 11: "k_layer_att", 12: "k_ffn", 13: "k_layer"}
PRESETS = {2: "MioTTS-0.1B Q8_0", 3: "MioTTS-1.7B Q4_K_M", 4: "MioTTS-2.6B Q8_0",
           6: "MioTTS-2.6B Q8_0 (LFM2 shape: 22 short-conv + 8 attention layers)", 12: "MioTTS-1.7B BF16"}
PROMPT = "こんにちは、今日はいい天気ですね。"  # README.md:83, SURVEY 8(d)


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--preset", type=int, default=3, choices=sorted(PRESETS))
    p.add_argument("--tokens", type=int, default=700)
    p.add_argument("--utts-per-step", type=int, default=1,
                   help="single-utterance syntheses per step, one after another")
    p.add_argument("--utts-per-gpu", type=int, default=1,
                   help="B > 1: each step decodes B utterances together per GPU (batched engine)")
    p.add_argument("--workdir", default=os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench"))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-tokens", type=int, default=64)
    p.add_argument("--no-cpu-c1", action="store_true", help="skip the C1 leg (0.1B Q8_0 CPU utterance)")
    p.add_argument("--cpu-codes", type=int, default=40)
    p.add_argument("--batch", type=int, default=8,
                   help="also time B utterances decoded together per GPU (N=1 only; 0 = skip)")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--no-configs", action="store_true",
                   help="skip the other BASELINE config lines (C2, C4 on both 2.6B shapes, C5) a default N=1 run adds")
    p.add_argument("--launcher-selftest", action="store_true",
                   help="tests only: the launcher + timed region with a CPU sleep as the utterance, no GPU; "
                        "prints a 'launcher self-test' line, never the metric")
    return p.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """N fresh child processes of this script, one per GPU (rank i on LOCAL_RANK i), started
    before this process has touched the GPU; returns the worst child exit status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def prompt_tokens(text: str):
    """normalize_tts_text + build_prompt + tokenize with the synthetic byte-level vocab
    (test-to-speech.cpp:90-92,114-125): specials -> ids 256/257/258, bytes -> ids 0..255."""
    import miotts_amd as m
    norm = m.normalize_text(text)
    toks = [256, 257] + list("user\n".encode()) + list(norm.encode("utf-8")) + [258]
    toks += list("\n".encode()) + [257] + list("assistant\n".encode())
    return toks


def ensure_files(workdir, preset, rank, barrier):
    import miotts_amd as m
    os.makedirs(workdir, exist_ok=True)
    llm = os.path.join(workdir, f"llm_preset{preset}.gguf")
    codec = os.path.join(workdir, "miocodec_synth.gguf")
    voice = os.path.join(workdir, "voice_synth.emb.gguf")
    if rank == 0:
        for path, fn in ((llm, lambda p: m.synth_llm(p, preset, 1)), (codec, lambda p: m.synth_codec(p, 0, 1)),
                         (voice, lambda p: m.synth_voice(p, 7))):
            if not os.path.exists(path):
                tmp = path + ".tmp"
                fn(tmp)
                os.replace(tmp, path)
    barrier()
    return llm, codec, voice


def cpu_baseline(llm_path, codec_path, voice_path, n_tok, n_codes, utt_tokens, threads):
    """The C oracle ("port") on `threads` OpenMP threads: n_tok decode steps at positions
    spread evenly over [0, utt_tokens) (attention cost grows with the position; the cache
    rows it reads hold zeros, which costs the same as real rows) + codec/iSTFT of n_codes,
    extrapolated to one utterance of utt_tokens tokens."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import miotts_amd as m
    import pyoracle
    prev = pyoracle.set_threads(threads)
    try:
        o = pyoracle.Llm(llm_path, utt_tokens + 8)
        positions = [int(p) for p in np.linspace(0, utt_tokens - 1, n_tok)]
        o.eval(m.SYNTH_SPEECH0, 0)  # warm (page in the weights)
        t0 = time.perf_counter()
        for i, pos in enumerate(positions):
            o.eval(m.SYNTH_SPEECH0 + (i * 97) % 12800, pos)
        t_tok = (time.perf_counter() - t0) / n_tok
        c = pyoracle.Codec(codec_path)
        emb = m.read_voice(voice_path)
        codes = (np.arange(n_codes) * 7919) % 12800
        t0 = time.perf_counter()
        c.decode_pcm(codes, emb)
        t_code = (time.perf_counter() - t0) / n_codes
    finally:
        pyoracle.set_threads(prev)
    wall = utt_tokens * t_tok + utt_tokens * t_code
    audio = utt_tokens * 1764 / 44100.0
    host = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = host
    return {"value": round(audio / wall, 4), "unit": "x realtime (audio s / wall s)", "cores": threads,
            "host_cpus": host, "affinity_cpus": affinity,
            "cores_note": f"{threads} OpenMP threads = this job's CPU share (OMP_NUM_THREADS, else min(16, host "
                          f"CPUs)); the host reports {host} CPUs ({affinity} in this process's affinity mask)",
            "kind": "port",
            "sample": f"oracle decode of {n_tok} tokens at positions 0..{utt_tokens - 1} "
                      f"({t_tok * 1e3:.1f} ms/token) + codec+iSTFT of {n_codes} codes "
                      f"({t_code * 1e3:.2f} ms/code), extrapolated to {utt_tokens} tokens"}


def cpu_baseline_c1(workdir, tokens, threads):
    """BASELINE configs[0] (C1: MioTTS-0.1B Q8_0, the CPU path of miotts-stream-benchmark,
    stream-benchmark.cpp:148-166): one whole utterance through the C oracle ("port"; the
    reference's own CPU path needs the absent ggml) on `threads` OpenMP threads,
    NOT extrapolated: the chat-template prompt prefilled token by token, `tokens` sampled speech
    tokens, MioCodec + iSTFT of the codes, timed end to end (tools/cpu_full.py's run)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import miotts_amd as m
    import pyoracle
    llm_path, codec_path, voice_path = ensure_files(workdir, 2, 0, lambda: None)
    prompt = prompt_tokens(PROMPT)
    allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
    prev = pyoracle.set_threads(threads)
    try:
        o = pyoracle.Llm(llm_path, len(prompt) + tokens + 8)
        c = pyoracle.Codec(codec_path)
        emb = m.read_voice(voice_path)
        o.eval(prompt[0], 0)  # page the weights in (not timed)
        o.reset()
        t0 = time.perf_counter()
        ids = o.generate(prompt, tokens, 0.8, 42, allow=allow)
        t1 = time.perf_counter()
        pcm = c.decode_pcm(np.asarray(ids, np.int64) - m.SYNTH_SPEECH0, emb)
        t2 = time.perf_counter()
    finally:
        pyoracle.set_threads(prev)
    audio = pcm.size / 44100.0
    return {"value": round(audio / (t2 - t0), 4), "unit": "x realtime (audio s / wall s)", "cores": threads,
            "kind": "port", "model": PRESETS[2], "tokens": len(ids), "prompt_tokens": len(prompt),
            "llm_s": round(t1 - t0, 3), "codec_istft_s": round(t2 - t1, 3), "wall_s": round(t2 - t0, 3),
            "sample": f"one whole utterance, not extrapolated: {len(prompt)}-token prompt + {len(ids)} tokens "
                      f"+ codec/iSTFT of {len(ids)} codes ({audio:.1f} s audio)"}


def eos_tail(llm, prompt, tokens_per_step_us):
    """Cost of the decode steps queued past an end token (test-to-speech.cpp:168-170 breaks
    before the next llama_decode): an EOS-ending run (1 in 4 allowed ids is the end token,
    temperature 2), then mio_hip_llm_tail: steps issued after the end token and the GPU time of
    the step graphs queued after the one that sampled it (the host stops issuing graphs when the
    sampler's mapped host word says so)."""
    import miotts_amd as m
    for seed in range(11, 40):
        toks = llm.generate(prompt, 400, 2.0, seed, allow=(m.SYNTH_EOT, m.SYNTH_SPEECH0 + 3),
                            eos=(m.SYNTH_EOT, m.SYNTH_IM_END), check_interval=32)
        wasted, timed, ms = llm.tail()
        if timed:
            break
    r = {"tokens_before_eos": len(toks), "steps_after_eos": wasted, "timed_steps": timed,
         "timed_ms": round(ms, 3), "stop": "end-token host word, step graphs of 8, 2 queued ahead"}
    if timed:
        # every post-EOS step, at the timed steps' cost: the whole tail's GPU time
        r["tail_ms_est"] = round(ms / timed * wasted, 3)
    if timed:
        r["us_per_step_after_eos"] = round(ms * 1e3 / timed, 2)
        r["us_per_step_decoding"] = round(tokens_per_step_us, 2)
        r["launches_per_step"] = len(llm.step_kinds())
    return r


def batched_line(a, llm, codec, dev, prompt, allow, d_emb, d_pcm):
    """B utterances per GPU decoded together (mio_hip_llm_generate_batch: one weight pass per
    step for all B), then each through MioCodec + iSTFT into HBM. Reported beside `value`
    (which stays the single-utterance workload BASELINE's metric is quoted on)."""
    B = a.batch
    step = make_batch_step(a.tokens, B, llm, codec, dev, prompt, allow, d_emb, d_pcm)
    step(0, False)  # warm (graph capture)
    dev.sync()
    t0 = time.perf_counter()
    samples, llm_s, _, _ = step(5000, True)
    wall = time.perf_counter() - t0
    return {"utterances": B, "value": round(samples / codec.sample_rate / wall, 3),
            "unit": "x realtime (audio s / wall s), aggregate of the B utterances on one GPU",
            "llm_ms": round(llm_s * 1e3, 3), "llm_ms_per_step": round(llm_s * 1e3 / a.tokens, 4),
            "codec_istft_ms": round((wall - llm_s) * 1e3, 3), "wall_ms": round(wall * 1e3, 3)}


def make_batch_step(tokens, B, llm, codec, dev, prompt, allow, d_emb, d_pcm):
    """One step of B utterances decoded together, then their codec + iSTFT decodes run
    concurrently (mio_hip_codec_decode_pcm_batch: up to 3 streams, each with its own workspace;
    PCM left in HBM). step(seed_base, _) -> (audio samples, llm seconds, codec+iSTFT ms, 0)."""
    import numpy as np
    import miotts_amd as m
    d_outs = [dev.empty((tokens * codec.samples_per_token,), np.float32) for _ in range(B)]

    def step(seed_base, _record):
        seeds = [utterance_seed(0, seed_base + b) for b in range(B)]
        t0 = time.perf_counter()
        outs = llm.generate_batch([prompt] * B, tokens, 0.8, seeds, allow=allow, check_interval=64)
        t1 = time.perf_counter()
        for toks in outs:
            if len(toks) != tokens:
                raise RuntimeError("batched utterance ended early")
        d_codes = [dev.upload((toks - m.SYNTH_SPEECH0).astype(np.int32)) for toks in outs]
        lens = codec.decode_pcm_batch_device(d_codes, [len(t) for t in outs], d_emb, d_outs)
        c_ms, _ = codec.last_timings()
        dev.sync()
        return sum(lens), t1 - t0, c_ms, 0.0

    return step


def baseline_configs(a, llm_path, codec_path, voice_path):
    """The other BASELINE.json configs, each in a child process after the timed region (N=1,
    rank 0): C2 (0.1B Q8_0, one utterance per step), C4 per GPU (2.6B Q8_0, 8 utterances decoded
    together; the plain-attention stand-in and the LFM2-2.6B shape), and C5 (the streaming
    benchmark CLI, miotts-stream-benchmark, 1.7B Q4_K_M, 700 tokens: test-to-speech.cpp:435-614).
    Each is this script's own timed region (or the CLI's own clock) at short K; a failure is
    recorded in its entry and never touches the headline line."""
    import re
    import subprocess
    res = {}
    me, py = os.path.abspath(__file__), sys.executable
    common = ["--no-cpu-baseline", "--batch", "0", "--no-roofline", "--no-configs", "--workdir", a.workdir,
              "--tokens", str(a.tokens)]
    runs = {"C2_0p1b_q8_single": ["--preset", "2", "--steps", "3", "--warmup", "1"],
            "C4_2p6b_q8_8_per_gpu": ["--preset", "4", "--utts-per-gpu", "8", "--steps", "1", "--warmup", "1"],
            "C4_2p6b_lfm2_8_per_gpu": ["--preset", "6", "--utts-per-gpu", "8", "--steps", "1", "--warmup", "1"]}
    for name, args in runs.items():
        t0 = time.perf_counter()
        try:
            p = subprocess.run([py, me] + args + common, capture_output=True, text=True, timeout=400)
            line = json.loads(p.stdout.strip().splitlines()[-1])
            res[name] = {"value": line["value"], "unit": line["unit"], "ms_per_step": line["ms_per_step"],
                         "steps": line["steps"], "config": line["config"], "stage_ms": line.get("stage_ms"),
                         "child_wall_s": round(time.perf_counter() - t0, 1)}
        except Exception as e:  # noqa: BLE001 - reported, the headline line stands
            res[name] = {"error": repr(e)[:400]}
    t0 = time.perf_counter()
    try:
        exe = os.path.join(REPO, "miotts-llama.cpp_amd", "build", "miotts-stream-benchmark")
        p = subprocess.run([exe, "-m", llm_path, "-c", codec_path, "-v", voice_path, "-p", PROMPT, "--max-tokens",
                            str(a.tokens), "--speech-only", "--ignore-eos"], capture_output=True, text=True, timeout=300)
        kv = {k: float(v) for k, v in re.findall(r"^stream_bench\.([\w.]+)=([-\d.eE+]+)", p.stdout, re.M)}
        res["C5_stream_1p7b"] = {"value": round(kv["x_realtime"], 3), "unit": "x realtime (audio s / wall s)",
                                 "stream_bench": kv, "child_wall_s": round(time.perf_counter() - t0, 1),
                                 "config": {"workload": "miotts-stream-benchmark, 1.7B Q4_K_M synthetic, "
                                                        f"{a.tokens} speech tokens, 20-token checks"}}
    except Exception as e:  # noqa: BLE001
        res["C5_stream_1p7b"] = {"error": repr(e)[:400]}
    return res


def utterance_seed(rank: int, index: int) -> int:
    """Distinct sampler seed per (rank, utterance index): ranks never replay each other's work."""
    return 42 + 7919 * rank + 104729 * index


def timed_region(warmup, steps, utts_per_step, rank, utterance, sync, barrier, dist):
    """Weak-scaling timed region shared by every rank (no data-path collective): W untimed
    warmup steps, then K steps bracketed by barrier + device sync on both sides. Returns
    (max elapsed over ranks, sum of audio samples over ranks); the only collectives are
    these two scalar reductions after the clock has stopped."""
    for w in range(warmup):
        for u in range(utts_per_step):
            utterance(utterance_seed(rank, w * utts_per_step + u), False)
    sync()
    barrier()
    t_start = time.perf_counter()
    samples = 0
    for s in range(steps):
        for u in range(utts_per_step):
            samples += utterance(utterance_seed(rank, 1000 + s * utts_per_step + u), True)
    sync()
    barrier()
    elapsed = time.perf_counter() - t_start
    if dist is None:
        return elapsed, float(samples)
    return all_reduce(dist, elapsed, "max"), all_reduce(dist, float(samples), "sum")


def all_reduce(dist, v: float, op: str) -> float:
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def roofline(llm, preset):
    """Dominant decode-step kernel by in-graph time per token (step timeline) with its
    algorithmic bytes; see the module docstring."""
    import numpy as np
    tl = llm.timeline()
    nl = tl.shape[0]
    # the step's launches in order (layer kinds, then lm_head); the sampler runs inside layer
    # 0's first launch
    step = llm.step_kinds()
    assert len(step) == nl, (len(step), nl)
    names = [KERNEL_NAMES[k] for k in step]
    fused = 10 in step or 11 in step or 13 in step
    dur = np.nanmax(tl[:, :, 7], axis=1) - np.nanmin(tl[:, :, 0], axis=1)
    step_wall_us = float(np.nanmax(tl[-1, :, 7]) - np.nanmin(tl[0, :, 0]))
    per_kernel = {}
    for i, nm in enumerate(names):
        per_kernel.setdefault(nm, []).append(float(dur[i]))
    bytes_of, event_us = {}, {}
    for which in sorted(set(step)):
        ms, by = llm.time_kernel(which, 40)
        bytes_of[KERNEL_NAMES[which]] = by
        event_us[KERNEL_NAMES[which]] = ms * 1e3
    dom = max(bytes_of, key=lambda k: sum(per_kernel[k]))
    dom_us = float(np.mean(per_kernel[dom]))
    # achieved: HIP events around back-to-back launches of the kernel on its own stream (the
    # timeline's in-graph span runs the diagnostic instantiation: reported beside it)
    achieved = bytes_of[dom] / (event_us[dom] * 1e-6) / 1e9
    step_bytes = sum(bytes_of[KERNEL_NAMES[k]] for k in step)
    step_gbs = step_bytes / (step_wall_us * 1e-6) / 1e9
    traffic = None
    tfile = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        try:
            tj = json.load(open(tfile))
            if tj.get("preset") == preset:
                traffic = tj.get("per_launch_bytes", {}).get(dom)
        except Exception:
            traffic = None
    return {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "bytes_per_launch": bytes_of[dom],
            "avg_launch_us": round(event_us[dom], 3), "in_graph_avg_launch_us": round(dom_us, 3),
            "frac_in_graph": round(bytes_of[dom] / (dom_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "event_us_all": {k: round(v, 3) for k, v in event_us.items()},
            "step_bytes": step_bytes, "step_graph_wall_us": round(step_wall_us, 1),
            "step_achieved_GBps": round(step_gbs, 1), "step_frac": round(step_gbs / HBM_PEAK_GBS, 4),
            "step_weight_bytes": llm.weight_bytes(),
            "per_token_us": {k: round(sum(v), 1) for k, v in per_kernel.items()},
            "bytes_per_launch_all": bytes_of, "launches_per_step": nl,
            "note": ("timeline, events and attention bytes at decode position ~400 (as the PMC run)"
                     + ("; k_att_o = attention + O projection in one launch (layer 0; bytes: K/V rows, q|k|v, "
                        "chunk records, W_o, x), k_layer_att = RMSNorm + q|k|v + attention + O in one launch "
                        "(layers >= 1; + W_q|k|v), k_layer = k_layer_att + the FFN pair in one launch (layers >= 1; "
                        "+ W_gate|up, W_down, h); their event times exclude the counter reset a step's next "
                        "launch does" if fused else ""))}


F32_MFMA_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: f32 matrix (and vector) peak, exact f32


def codec_roofline(flops, codec_ms, tokens):
    """The codec's compute roofline: its algorithmic FLOPs (every GEMM, conv and
    banded-attention product it issues, mio_hip_codec_last_flops) over its event-timed time
    against the f32 MFMA peak; with the PMC run's MFMA-busy share when profiles hold one."""
    tfs = flops / (codec_ms * 1e-3) / 1e12
    r = {"bound": "mfma", "flops": round(flops), "ms": round(codec_ms, 3), "achieved": round(tfs, 2),
         "peak": F32_MFMA_PEAK_TFS, "unit": "TFLOP/s", "frac": round(tfs / F32_MFMA_PEAK_TFS, 4),
         "codes": tokens, "mfma_busy": None}
    f = os.path.join(REPO, "profiles", "pmc_codec_mfma.json")
    if os.path.exists(f):
        try:
            r["mfma_busy"] = json.load(open(f)).get("mfma_busy_frac")
        except Exception:
            pass
    return r


def main():
    argv = sys.argv[1:]
    a = parse_args(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a.gpus, argv))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        if dist is not None:
            dist.barrier()

    if a.launcher_selftest:  # tests/test_bench_dist.py: the N-rank launcher without a GPU
        def fake(seed, record):
            time.sleep(0.02 * (rank + 1))
            return 1000
        elapsed, samples = timed_region(a.warmup, a.steps, a.utts_per_step, rank, fake, lambda: None, barrier, dist)
        if rank == 0:
            print(json.dumps({"metric": "launcher self-test", "n_gpus": world, "samples": samples,
                              "elapsed": elapsed, "pid_rank0": os.getpid(),
                              "local_rank": local_rank}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    import numpy as np
    import miotts_amd as m

    llm_path, codec_path, voice_path = ensure_files(a.workdir, a.preset, rank, barrier)
    n_dev = m.device_count()
    dev = m.Device(local_rank % n_dev)  # ranks share a GPU only when there are fewer GPUs than ranks
    t_load = time.perf_counter()
    llm = m.Llm(dev, llm_path, 2048)
    t_llm = time.perf_counter()
    codec = m.Codec(dev, codec_path)
    load = {"llm_ms": round(llm.load_ms(), 1), "llm_wall_ms": round((t_llm - t_load) * 1e3, 1),
            "codec_wall_ms": round((time.perf_counter() - t_llm) * 1e3, 1), "llm_bytes": llm.weight_bytes()}
    emb = m.read_voice(voice_path)
    prompt = prompt_tokens(PROMPT)
    allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)

    stage = {"llm_ms": 0.0, "codec_ms": 0.0, "istft_ms": 0.0, "codec_wall_ms": 0.0}
    codec_flops = []

    d_emb = dev.upload(np.ascontiguousarray(emb, np.float32))
    d_pcm = dev.empty((a.tokens * codec.samples_per_token,), np.float32)
    B = a.utts_per_gpu

    def utterance(seed, record):
        t0 = time.perf_counter()
        toks = llm.generate(prompt, a.tokens, 0.8, seed, allow=allow, check_interval=32)
        t1 = time.perf_counter()
        d_codes = dev.upload((toks - m.SYNTH_SPEECH0).astype(np.int32))
        n = codec.decode_pcm_device(d_codes, len(toks), d_emb, d_pcm)
        dev.sync()
        t2 = time.perf_counter()
        if record:
            c_ms, i_ms = codec.last_timings()
            stage["llm_ms"] += (t1 - t0) * 1e3
            stage["codec_wall_ms"] += (t2 - t1) * 1e3
            stage["codec_ms"] += c_ms
            stage["istft_ms"] += i_ms
            codec_flops.append(codec.last_flops())
        if len(toks) != a.tokens or n != a.tokens * codec.samples_per_token:
            raise RuntimeError(f"utterance produced {len(toks)} tokens / {n} samples")
        return n

    batch_llm_s = []
    if B > 1:
        bstep = make_batch_step(a.tokens, B, llm, codec, dev, prompt, allow, d_emb, d_pcm)

        def step_fn(seed, record):
            samples, llm_s, c_ms, i_ms = bstep(seed * 131, record)
            if record:
                # whole-step totals; divided by the utterances (steps * B) below: per utterance,
                # the batched decode's wall is shared by its B utterances
                stage["llm_ms"] += llm_s * 1e3
                stage["codec_ms"] += c_ms
                stage["istft_ms"] += i_ms
                batch_llm_s.append(llm_s)
            return samples
        utts = 1
    else:
        step_fn, utts = utterance, a.utts_per_step

    elapsed, total_samples = timed_region(a.warmup, a.steps, utts, rank, step_fn, dev.sync, barrier, dist)
    audio_s = total_samples / codec.sample_rate
    value = audio_s / elapsed
    utt_per_rank = a.steps * (B if B > 1 else a.utts_per_step)

    # PCIe-inclusive: each rank copies its utterances' PCM to host memory (ranks in parallel:
    # the slowest rank's copy time counts, never `value`)
    t0 = time.perf_counter()
    for _ in range(3):
        d_pcm.numpy()
    d2h_s = all_reduce(dist, (time.perf_counter() - t0) / 3, "max")
    value_pcie = audio_s / (elapsed + d2h_s * utt_per_rank)

    # WAV epilogue on the device (mio_hip_pcm_finish: peak normalise + PCM16) of the last
    # utterance, HIP events on the device stream; reported beside the stage times
    n_pcm = a.tokens * codec.samples_per_token
    d_pcm16 = dev.empty((n_pcm,), np.int16)
    lib = m.lib()
    pf_ms = []
    for _ in range(4):
        dev.mark(14)
        m.check(lib.mio_hip_pcm_finish(dev.h, d_pcm.ptr, n_pcm, 1, d_pcm16.ptr, None, None))
        dev.mark(15)
        dev.sync()
        pf_ms.append(dev.elapsed_ms(14, 15))
    pcm_finish_ms = round(min(pf_ms[1:]), 4)

    roof = None
    if rank == 0 and not a.no_roofline and B == 1:
        # roofline at decode position ~400, the utterance's mean attention length and the
        # position of the PMC passes (tools/pmc_run.py)
        llm.generate(prompt, max(1, ROOF_POS + 2 - len(prompt)), 0.8, 7, allow=allow, check_interval=1000)
        roof = roofline(llm, a.preset)
    tail = None
    if rank == 0 and B == 1 and stage["llm_ms"] > 0:
        tail = eos_tail(llm, prompt, stage["llm_ms"] / utt_per_rank / a.tokens * 1e3)

    steps_total = utt_per_rank
    model = PRESETS[a.preset]
    out = {
        # BASELINE.json's metric (quoted on preset 3); other presets name their own model
        "metric": "realtime factor (audio s / wall s) + stage ms llm/codec/istft, " + model.replace("MioTTS-", ""),
        "value": round(value, 3),
        "unit": "x realtime (audio s / wall s)",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("int8-dot (q8_0 x q8_0)" if "Q8_0" in model
                  else ("bf16-dot2 (bf16 x bf16-rounded activation, f32 sums)" if "BF16" in model
                        else "int8-dot (q4_K/q6_K x q8_K)"))
                 + " + f32/f16 codec",
        "data": "synthetic",
        "config": {"workload": (f"{model} {'single utterance' if B == 1 else f'{B} utterances decoded together'}"
                                f", {a.tokens} speech tokens -> MioCodec -> iSTFT "
                                f"({a.tokens * 1764 / 44100:.1f} s audio each) per GPU"),
                   "model": model, "global_batch": world * (B if B > 1 else a.utts_per_step),
                   "seq_len": a.tokens, "parallelism": f"utterance-sharded x{world} (no collective)",
                   "devices_visible": n_dev},
        "load_ms": load,
        "stage_ms": {**{k: round(v / steps_total, 3) for k, v in stage.items()},
                     "pcm_finish_ms": pcm_finish_ms},
        "llm_ms_per_token": round(stage["llm_ms"] / steps_total / a.tokens, 4),
        "roofline": roof,
        "value_pcie_inclusive": round(value_pcie, 3),
        "cpu_baseline": None,
        "eos_tail": tail,
    }
    if codec_flops and stage["codec_ms"] > 0:
        out["codec_roofline"] = codec_roofline(sum(codec_flops) / len(codec_flops), stage["codec_ms"] / steps_total,
                                               a.tokens)
    if B > 1 and batch_llm_s:
        # the batched decode step against its weight stream: one weight pass per step serves
        # the B utterances (+ each one's K/V rows at the mean position)
        step_s = sum(batch_llm_s) / len(batch_llm_s) / a.tokens
        info = llm.n_layer, llm.n_kv, llm.head_dim
        kv = 2 * 2 * info[0] * info[1] * info[2] * (len(prompt) + a.tokens // 2) * B
        by = llm.weight_bytes() + kv
        out["batched_step"] = {"utterances": B, "ms_per_step": round(step_s * 1e3, 4),
                               "bytes_per_step": by, "achieved_GBps": round(by / step_s / 1e9, 1),
                               "step_frac": round(by / step_s / 1e9 / HBM_PEAK_GBS, 4),
                               "note": "decode steps incl. the prompt prefill; bytes = weights + K/V rows "
                                       "of B streams at the mean position"}
    if world == 1 and a.batch > 0 and B == 1:
        out["batched"] = batched_line(a, llm, codec, dev, prompt, allow, d_emb, d_pcm)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        share = int(os.environ.get("OMP_NUM_THREADS", 0) or min(16, os.cpu_count() or 1))
        out["cpu_baseline"] = cpu_baseline(llm_path, codec_path, voice_path, a.cpu_tokens, a.cpu_codes, a.tokens,
                                           share)
        out["cpu_baseline_4_threads"] = cpu_baseline(llm_path, codec_path, voice_path, max(16, a.cpu_tokens // 4),
                                                     a.cpu_codes // 2, a.tokens, 4)
        if not a.no_cpu_c1:
            out["cpu_baseline_c1"] = cpu_baseline_c1(a.workdir, a.tokens, share)
    if rank == 0 and world == 1 and B == 1 and not a.no_configs:
        out["baseline_configs"] = baseline_configs(a, llm_path, codec_path, voice_path)
    if rank == 0:
        print(json.dumps(out, ensure_ascii=False), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
