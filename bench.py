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

Multi-GPU: one process per GPU (torchrun), each rank synthesizes its own utterances
(utterances are independent: no collective on the data path, "scaling": "weak"); a gloo
barrier brackets the timed region and the max elapsed over ranks is used.

roofline: the dominant decode-step kernel (largest time per token), timed inside the
captured step graph by the step timeline (first workgroup start -> last workgroup end of
every launch, s_memrealtime, mio_hip_llm_timeline) right after the timed region:
achieved = its algorithmic bytes per launch (GGUF bytes of the matrices it streams + its
activations) / mean launch duration; peak = 8 TB/s HBM3E. traffic = the same kernel's
HBM bytes per launch from rocprofv3 PMC (FETCH_SIZE x 2 on gfx950 + WRITE_SIZE,
profiles/pmc_traffic.json, tools/pmc_traffic.py). HIP-event timing of back-to-back
launches of the same kernel is reported as event_avg_launch_us (cache-warm).
cpu_baseline: the C oracle (oracle/, "port") on rank 0 at N=1 only, timed on a bounded
sample (decode steps + codec/iSTFT of a few codes) and extrapolated to one utterance.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
KERNEL_NAMES = {0: "k_attn_in", 1: "k_attention", 2: "k_attn_out", 3: "k_ffn_in", 4: "k_ffn_down",
                6: "k_lm_head"}
PRESETS = {2: "MioTTS-0.1B Q8_0", 3: "MioTTS-1.7B Q4_K_M", 4: "MioTTS-2.6B Q8_0"}
PROMPT = "こんにちは、今日はいい天気ですね。"  # README.md:83, SURVEY 8(d)


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--preset", type=int, default=3, choices=sorted(PRESETS))
    p.add_argument("--tokens", type=int, default=700)
    p.add_argument("--utts-per-step", type=int, default=1)
    p.add_argument("--workdir", default=os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench"))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-tokens", type=int, default=12)
    p.add_argument("--cpu-codes", type=int, default=40)
    p.add_argument("--batch", type=int, default=8,
                   help="also time B utterances decoded together per GPU (N=1 only; 0 = skip)")
    return p.parse_args()


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


def cpu_baseline(llm_path, codec_path, voice_path, n_tok, n_codes, utt_tokens):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import miotts_amd as m
    import pyoracle
    o = pyoracle.Llm(llm_path, 256)
    t0 = time.perf_counter()
    for pos in range(n_tok):
        o.eval(m.SYNTH_SPEECH0 + (pos * 97) % 12800, pos)
    t_tok = (time.perf_counter() - t0) / n_tok
    c = pyoracle.Codec(codec_path)
    emb = m.read_voice(voice_path)
    codes = (np.arange(n_codes) * 7919) % 12800
    t0 = time.perf_counter()
    c.decode_pcm(codes, emb)
    t_code = (time.perf_counter() - t0) / n_codes
    wall = utt_tokens * t_tok + utt_tokens * t_code
    audio = utt_tokens * 1764 / 44100.0
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": round(audio / wall, 4), "unit": "x realtime (audio s / wall s)", "cores": cores,
            "kind": "port",
            "sample": f"oracle decode of {n_tok} tokens ({t_tok * 1e3:.1f} ms/token) + codec+iSTFT of "
                      f"{n_codes} codes ({t_code * 1e3:.2f} ms/code), extrapolated to {utt_tokens} tokens"}


def batched_line(a, llm, codec, dev, prompt, allow, d_emb, d_pcm):
    """B utterances per GPU decoded together (mio_hip_llm_generate_batch: one weight pass per
    step for all B), then each through MioCodec + iSTFT into HBM. Reported beside `value`
    (which stays the single-utterance workload BASELINE's metric is quoted on)."""
    import numpy as np
    import miotts_amd as m
    B = a.batch
    seeds = [utterance_seed(0, 5000 + b) for b in range(B)]
    llm.generate_batch([prompt] * B, a.tokens, 0.8, seeds, allow=allow)  # warm (graph capture)
    dev.sync()
    t0 = time.perf_counter()
    outs = llm.generate_batch([prompt] * B, a.tokens, 0.8, seeds, allow=allow, check_interval=64)
    t1 = time.perf_counter()
    samples = 0
    for toks in outs:
        d_codes = dev.upload((toks - m.SYNTH_SPEECH0).astype(np.int32))
        samples += codec.decode_pcm_device(d_codes, len(toks), d_emb, d_pcm)
    dev.sync()
    t2 = time.perf_counter()
    if any(len(t) != a.tokens for t in outs):
        raise RuntimeError("batched utterance ended early")
    wall = t2 - t0
    return {"utterances": B, "value": round(samples / codec.sample_rate / wall, 3),
            "unit": "x realtime (audio s / wall s), aggregate of the B utterances on one GPU",
            "llm_ms": round((t1 - t0) * 1e3, 3), "llm_ms_per_step": round((t1 - t0) * 1e3 / a.tokens, 4),
            "codec_istft_ms": round((t2 - t1) * 1e3, 3), "wall_ms": round(wall * 1e3, 3)}


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
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n = torch.tensor([samples], dtype=torch.float64)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    return float(t.item()), float(n.item())


def main():
    a = parse_args()
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

    import numpy as np
    import miotts_amd as m

    llm_path, codec_path, voice_path = ensure_files(a.workdir, a.preset, rank, barrier)
    dev = m.Device(local_rank)
    llm = m.Llm(dev, llm_path, 2048)
    codec = m.Codec(dev, codec_path)
    emb = m.read_voice(voice_path)
    prompt = prompt_tokens(PROMPT)
    allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)

    stage = {"llm_ms": 0.0, "codec_ms": 0.0, "istft_ms": 0.0, "codec_wall_ms": 0.0}

    d_emb = dev.upload(np.ascontiguousarray(emb, np.float32))
    d_pcm = dev.empty((a.tokens * codec.samples_per_token,), np.float32)

    def utterance(seed, record):
        t0 = time.perf_counter()
        toks = llm.generate(prompt, a.tokens, 0.8, seed, allow=allow, check_interval=20)
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
        if len(toks) != a.tokens or n != a.tokens * codec.samples_per_token:
            raise RuntimeError(f"utterance produced {len(toks)} tokens / {n} samples")
        return n

    elapsed, total_samples = timed_region(a.warmup, a.steps, a.utts_per_step, rank, utterance,
                                          dev.sync, barrier, dist)
    audio_s = total_samples / codec.sample_rate
    value = audio_s / elapsed

    # PCIe-inclusive: the PCM of one utterance copied to host memory (never `value`)
    t0 = time.perf_counter()
    for _ in range(3):
        d_pcm.numpy()
    d2h_s = (time.perf_counter() - t0) / 3
    value_pcie = audio_s / (elapsed + d2h_s * a.steps * a.utts_per_step * world)

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

    # roofline: dominant kernel inside the captured step graph (timeline), then HIP events
    tl = llm.timeline()
    nl = tl.shape[0]
    names = [KERNEL_NAMES[k] for k in (0, 1, 2, 3, 4)] * ((nl - 2) // 5) + [KERNEL_NAMES[6], "k_sample"]
    dur = np.nanmax(tl[:, :, 7], axis=1) - np.nanmin(tl[:, :, 0], axis=1)
    step_wall_us = float(np.nanmax(tl[-1, :, 7]) - np.nanmin(tl[0, :, 0]))
    per_kernel = {}
    for i, nm in enumerate(names):
        per_kernel.setdefault(nm, []).append(float(dur[i]))
    bytes_of = {}
    event_us = {}
    for which in (0, 1, 2, 3, 4, 6):
        ms, by = llm.time_kernel(which, 40)
        bytes_of[KERNEL_NAMES[which]] = by
        event_us[KERNEL_NAMES[which]] = ms * 1e3
    dom = max((k for k in bytes_of if bytes_of[k] > 0), key=lambda k: sum(per_kernel[k]))
    dom_us = float(np.mean(per_kernel[dom]))
    dom_bytes = bytes_of[dom]
    achieved = dom_bytes / (dom_us * 1e-6) / 1e9
    traffic = None
    tfile = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        try:
            tj = json.load(open(tfile))
            if tj.get("preset") == a.preset:
                traffic = tj.get("per_launch_bytes", {}).get(dom)
        except Exception:
            traffic = None

    steps_total = a.steps * a.utts_per_step
    out = {
        # BASELINE.json's metric (quoted on preset 3); other presets name their own model
        "metric": "realtime factor (audio s / wall s) + stage ms llm/codec/istft, "
                  + PRESETS[a.preset].replace("MioTTS-", ""),
        "value": round(value, 3),
        "unit": "x realtime (audio s / wall s)",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("int8-dot (q8_0 x q8_0)" if "Q8_0" in PRESETS[a.preset] else "int8-dot (q4_K/q6_K x q8_K)")
                 + " + f32/f16 codec",
        "data": "synthetic",
        "config": {"workload": f"{PRESETS[a.preset]} single utterance, {a.tokens} speech tokens -> "
                               f"MioCodec -> iSTFT ({a.tokens * 1764 / 44100:.1f} s audio) per GPU",
                   "model": PRESETS[a.preset], "global_batch": world * a.utts_per_step,
                   "seq_len": a.tokens, "parallelism": f"utterance-sharded x{world} (no collective)"},
        "stage_ms": {**{k: round(v / steps_total, 3) for k, v in stage.items()},
                     "pcm_finish_ms": pcm_finish_ms},
        "llm_ms_per_token": round(stage["llm_ms"] / steps_total / a.tokens, 4),
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "bytes_per_launch": dom_bytes,
                     "avg_launch_us": round(dom_us, 3),
                     "event_avg_launch_us": round(event_us[dom], 3),
                     "step_weight_bytes": llm.weight_bytes(),
                     "step_graph_wall_us": round(step_wall_us, 1),
                     "per_token_us": {k: round(sum(v), 1) for k, v in per_kernel.items()}},
        "value_pcie_inclusive": round(value_pcie, 3),
        "cpu_baseline": None,
    }
    if world == 1 and a.batch > 0:
        out["batched"] = batched_line(a, llm, codec, dev, prompt, allow, d_emb, d_pcm)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(llm_path, codec_path, voice_path, a.cpu_tokens, a.cpu_codes, a.tokens)
    if rank == 0:
        print(json.dumps(out, ensure_ascii=False), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
