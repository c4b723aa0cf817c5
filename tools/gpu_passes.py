#!/usr/bin/env python
"""Named GPU passes as one table (replaces the round-4 one-off `scripts/r4_gpu*.sh` files).

    python tools/gpu_passes.py --list
    python tools/gpu_passes.py PASS [--out gpurun_out/PASS] [--dry]

Run it as the `gpurun` command (`gpurun -- 'python tools/gpu_passes.py validate'`). Each pass is a
list of steps, executed in order under their own `timeout -k 10`, stopping at the first failure
(no retries; no GPU step after a fault, abort or time limit). A heartbeat file under the output
directory is touched every 30 s so a long pass is never taken for a hung one. Step kinds:

  pytest  a pytest selection (GPU tier flags added)
  run     one command; its last line is echoed
  ab      `rounds` interleaved repetitions of each arm (arms differ only by environment), the same
          box for A and B: box-to-box clock variance exceeds most single optimisations
  prof    `rocprofv3 --kernel-trace` of a command; the trace is summarised on the box
          (scripts/prof_window.py, scripts/step_breakdown.py, scripts/prof_streams.py) and the
          raw trace deleted, so only small files come back
  pmc     one `rocprofv3 --pmc` counter pass (within the per-block slot limits), summarised by
          scripts/pmc_summary_csv.py
  smoke   __graft_entry__.smoke()

Profiles cite `tools/gpu_passes.py <name>` as their reproduce line. This parent process never
touches the GPU.
"""
from __future__ import annotations

import argparse
import glob
import os
import shlex
import shutil
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FATAL = {124, 134, 137, 139, -6, -9, -11}

GEN8 = "python -u tools/bench_generate.py --modes graph --new 128"
GEN64 = GEN8 + " --batch 64 --prompt 512"
DPO = "python -u bench.py"
MIX_EP8 = DPO + " --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8 --ep-capacity 1.25"
L70 = DPO + " --model llama3-70b --steps 2 --warmup 1"


def pytest(sel, t=1000):
    return {"kind": "pytest", "sel": sel, "timeout": t}


def run(name, cmd, t=600, env=None):
    return {"kind": "run", "name": name, "cmd": cmd, "timeout": t, "env": env or {}}


def ab(name, cmd, arms, rounds=2, t=600):
    return {"kind": "ab", "name": name, "cmd": cmd, "arms": arms, "rounds": rounds, "timeout": t}


def prof(name, cmd, summaries, t=420, env=None):
    return {"kind": "prof", "name": name, "cmd": cmd, "summaries": summaries, "timeout": t, "env": env or {}}


def pmc(name, counters, cmd, kernels, t=170, summary_args=(), include=None):
    return {"kind": "pmc", "name": name, "counters": counters, "cmd": cmd, "kernels": kernels, "timeout": t,
            "summary_args": list(summary_args), "include": include}


SMOKE = {"kind": "smoke", "timeout": 300}
DPO_TABLES = [("breakdown", []), ("window", ["--window", "adamw", "--by-grid", "--top", "60"])]
DEC_TABLE = [("window", ["--by-grid", "--top", "30", "--per", "4096"])]
ATTN_P1 = ("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
           "SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE")
ATTN_P2 = "SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS GRBM_COUNT"

PASSES = {
    # ---- whole-tree validation (the driver's round-end tiers, then every headline number)
    "tier": [pytest("tests -m gpu"), SMOKE, run("bench", DPO)],
    "validate": [
        pytest("tests -m gpu"), SMOKE, run("bench", DPO),
        run("bench_force_pg", DPO + " --force-pg --steps 5 --warmup 2", 300),
        run("gen8", GEN8, 300), run("gen64", GEN64, 300),
        run("rlhf8", "python -u tools/bench_rlhf.py --batch 8", 400),
        run("rlhf64_micro8", "python -u tools/bench_rlhf.py --batch 64 --micro 8"),
        run("ppo_zero8", "python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8"),
        run("mixtral_ep8", MIX_EP8 + " --steps 3 --warmup 2"),
        run("mixtral_ep8_fp8", MIX_EP8 + " --fp8 --steps 3 --warmup 2"),
        run("mixtral_ep8_hot", MIX_EP8 + " --ep-hot --steps 3 --warmup 2"),
        run("gen8_fp8", GEN8 + " --weight-dtype fp8", 300), run("gen64_fp8", GEN64 + " --weight-dtype fp8", 300),
        run("rlhf8_fp8", "python -u tools/bench_rlhf.py --batch 8 --rollout-dtype fp8", 400),
        run("ppo_zero8_fp8", "python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8 --rollout-dtype fp8"),
    ],
    # the same, in two gpurun-sized halves (a call runs at most 20 minutes)
    "validate-a": [
        pytest("tests -m gpu"), SMOKE, run("bench", DPO), run("bench20", DPO + " --steps 20 --warmup 5", 400),
        run("bench_force_pg", DPO + " --force-pg --steps 5 --warmup 2", 300),
        run("gen8", GEN8, 300), run("gen64", GEN64, 300),
        run("rlhf8", "python -u tools/bench_rlhf.py --batch 8", 400),
        run("rlhf64_micro8", "python -u tools/bench_rlhf.py --batch 64 --micro 8"),
    ],
    "validate-b": [
        run("ppo_zero8", "python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8"),
        run("mixtral_ep8", MIX_EP8 + " --steps 3 --warmup 2"),
        run("mixtral_ep8_fp8", MIX_EP8 + " --fp8 --steps 3 --warmup 2"),
        run("mixtral_ep8_hot", MIX_EP8 + " --ep-hot --steps 3 --warmup 2"),
        run("gen8_fp8", GEN8 + " --weight-dtype fp8", 300), run("gen64_fp8", GEN64 + " --weight-dtype fp8", 300),
        run("rlhf8_fp8", "python -u tools/bench_rlhf.py --batch 8 --rollout-dtype fp8", 400),
        run("ppo_zero8_fp8", "python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8 --rollout-dtype fp8"),
    ],
    # ---- round 6
    # residual adds as the C input of the o / down GEMMs (norms read/write one tensor each)
    "r6-resid": [pytest("tests/test_kernels_gpu.py -k 'fused_residual or norm_fwd_bwd or fused_swiglu'", 300),
                 ab("fused_resid", DPO + " --steps 5 --warmup 2", {"on": {"DLA_FUSED_RESIDUAL": "1"},
                                                                   "off": {"DLA_FUSED_RESIDUAL": "0"}}, 2, 300),
                 prof("dpo", DPO + " --steps 2 --warmup 1", DPO_TABLES)],
    # Q-only RoPE on load (rope kernel over K only) vs the q + k rope pass
    "r6-rope": [pytest("tests/test_kernels_gpu.py -k 'qkv_attention or rope or persistent or forced_rescale or fused_rope'", 400),
                ab("rope_qload", DPO + " --steps 5 --warmup 2", {"qload": {"DLA_ROPE_Q_ON_LOAD": "1"},
                                                                "qkpass": {"DLA_ROPE_Q_ON_LOAD": "0"}}, 2, 300),
                prof("dpo", DPO + " --steps 2 --warmup 1", DPO_TABLES)],
    # RLHF / PPO update costs: the forced one-rank RCCL path vs plain (reinforce update), and the
    # PPO update's kernels in issue order
    "r6-rlhf": [prof("rlhf_plain", "python -u tools/bench_rlhf.py --batch 8 --steps 2 --warmup 1",
                     [("window", ["--window", "adamw", "--by-grid", "--top", "40"]),
                      ("window", ["--window", "adamw", "--seq=-1500:1500"])], 500),
                prof("rlhf_forced", "python -u tools/bench_rlhf.py --batch 8 --force-pg --steps 2 --warmup 1",
                     [("window", ["--window", "adamw", "--by-grid", "--top", "40"]),
                      ("window", ["--window", "adamw", "--seq=-1500:1500"]), ("streams", ["--window", "adamw"])], 500),
                prof("ppo", "python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8 --steps 1 --warmup 1",
                     [("window", ["--by-grid", "--top", "50"]), ("window", ["--seq=-6000:6000"])], 500)],
    # LM-head dlogits^T written by the logprob backward kernel vs in-place kernel + transpose
    "r6-lpt": [pytest("tests/test_kernels_gpu.py tests/test_decode_gpu.py", 900),
               ab("logprob_t", DPO + " --steps 5 --warmup 2", {"on": {"DLA_LOGPROB_T": "1"},
                                                              "off": {"DLA_LOGPROB_T": "0"}}, 2, 300),
               prof("dpo", DPO + " --steps 2 --warmup 1", DPO_TABLES)],
    # forced-comm RLHF update after the shard-zeroing and C != D selection fixes: plain and forced
    # interleaved on one box, then the PPO update at the 8-rank ZeRO-1 shape
    "r6-rlhf2": [run("rlhf_plain0", "python -u tools/bench_rlhf.py --batch 8", 400),
                 run("rlhf_forced0", "python -u tools/bench_rlhf.py --batch 8 --force-pg", 400),
                 run("rlhf_plain1", "python -u tools/bench_rlhf.py --batch 8", 400),
                 run("rlhf_forced1", "python -u tools/bench_rlhf.py --batch 8 --force-pg", 400),
                 pytest("tests/test_ppo_shape.py tests/test_engines_gpu.py tests/test_distributed_gpu.py", 600),
                 run("dpo_plain", DPO + " --steps 5 --warmup 2", 300),
                 run("dpo_force_pg", DPO + " --force-pg --steps 5 --warmup 2", 300),
                 ab("ppo_critic_stream", "python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8",
                    {"side": {"DLA_PPO_CRITIC_STREAM": "1"}, "one": {"DLA_PPO_CRITIC_STREAM": "0"}}, 1, 500),
                 prof("rlhf_forced", "python -u tools/bench_rlhf.py --batch 8 --force-pg --steps 2 --warmup 1",
                      [("window", ["--window", "adamw", "--by-grid", "--top", "40"]), ("streams", ["--window", "adamw"])], 500)],
    # Llama-3-70B meshes on one build: 8x1 ZeRO-3 with full recompute and an 8-pair micro-batch;
    # 1x8 TP on the real one-rank RCCL group (per-rank shard shapes) vs the ShapeGroup stand-in;
    # 2x4; then an 8-layer TP stack under a kernel trace for the comm-stream overlap table
    "r6-70b": [run("zero3_8x1_recompute", L70 + " --zero 3 --fsdp-shape 8 --micro-pairs 8 --accum 2 --grad-ckpt full", 900),
               run("tp8_forced", L70 + " --tp-shape 8 --force-pg --micro-pairs 2 --accum 8", 600),
               run("tp8_shape", L70 + " --tp-shape 8 --micro-pairs 2 --accum 8", 600),
               run("fsdp2_tp4", L70 + " --zero 3 --fsdp-shape 2 --tp-shape 4 --micro-pairs 2 --accum 8", 600),
               prof("tp8_forced_stack", L70 + " --tp-shape 8 --force-pg --micro-pairs 2 --accum 8 --layers 8",
                    [("streams", ["--window", "adamw"]), ("window", ["--window", "adamw", "--by-grid", "--top", "30"])], 500),
               prof("tp8seq_forced_stack", L70 + " --tp-shape 8 --tp-seq --force-pg --micro-pairs 2 --accum 8 --layers 8",
                    [("streams", ["--window", "adamw"]), ("window", ["--window", "adamw", "--by-grid", "--top", "30"])], 500)],
    # Mixtral-8x7B on one build: EP 8 balanced vs the hot-expert rank (interleaved), EP 4 x EDP 2
    # bf16 / fp8, and the hot / balanced pair at capacity 1.125
    "r6-mixtral": [run("ep8_bal0", MIX_EP8 + " --steps 3 --warmup 2", 500),
                   run("ep8_hot0", MIX_EP8 + " --ep-hot --steps 3 --warmup 2", 500),
                   run("ep8_bal1", MIX_EP8 + " --steps 3 --warmup 2", 500),
                   run("ep8_hot1", MIX_EP8 + " --ep-hot --steps 3 --warmup 2", 500),
                   run("ep4_edp2", DPO + " --model mixtral-8x7b --ep-shape 4 --edp-shape 2 --micro-pairs 2 --accum 8"
                       " --ep-capacity 1.25 --steps 3 --warmup 2", 500),
                   run("ep4_edp2_fp8", DPO + " --model mixtral-8x7b --ep-shape 4 --edp-shape 2 --micro-pairs 2 --accum 8"
                       " --ep-capacity 1.25 --fp8 --steps 3 --warmup 2", 500),
                   run("ep8_bal_cf1125", DPO + " --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8"
                       " --ep-capacity 1.125 --steps 3 --warmup 2", 500),
                   run("ep8_hot_cf1125", DPO + " --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8"
                       " --ep-capacity 1.125 --ep-hot --steps 3 --warmup 2", 500),
                   prof("ep8_hot", MIX_EP8 + " --ep-hot --steps 2 --warmup 1",
                        [("window", ["--window", "adamw", "--by-grid", "--top", "40"])], 500),
                   prof("ep8_bal", MIX_EP8 + " --steps 2 --warmup 1",
                        [("window", ["--window", "adamw", "--by-grid", "--top", "40"])], 500)],
    # B = 8 decode attention at the RLHF shape (prompt 512 + 256 new: 6 key chunks): one-chunk
    # kernel + combine launch vs the loop kernel with the in-kernel combine (2 or 1 chunks/block)
    "r6-decode-combine": [ab("dec_rlhf_shape", "python -u tools/bench_generate.py --modes graph --prompt 512 --new 256",
                             {"base": {}, "loop2": {"DLA_DECODE_LOOP_MIN": "1"},
                              "loop1": {"DLA_DECODE_LOOP_MIN": "1", "DLA_DECODE_BLOCKS": "384"}}, 2, 300)],
    # the hot-expert rank at capacity 1.125, library rows adaptive vs static, under a kernel trace
    "r6-mixtral-cf": [prof("hot_cf1125_adaptive", DPO + " --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8"
                           " --ep-capacity 1.125 --ep-hot --steps 2 --warmup 1",
                           [("window", ["--window", "adamw", "--by-grid", "--top", "40"])], 500),
                      prof("hot_cf1125_static", DPO + " --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8"
                           " --ep-capacity 1.125 --ep-hot --steps 2 --warmup 1",
                           [("window", ["--window", "adamw", "--by-grid", "--top", "40"])], 500,
                           {"DLA_EP_ADAPTIVE_MAIN": "0"})],
    # round-6 decode default (fused-combine loop kernel at 1-2 chunks per block) and the adaptive
    # expert rows as tuned base + extension GEMMs
    "r6-check": [pytest("tests/test_decode_gpu.py tests/test_moe_gpu.py", 600),
                 run("gen_rlhf_shape", "python -u tools/bench_generate.py --modes graph --prompt 512 --new 256", 300),
                 run("rlhf8", "python -u tools/bench_rlhf.py --batch 8", 400),
                 run("ep8_hot", MIX_EP8 + " --ep-hot --steps 3 --warmup 2", 500),
                 run("ep8_bal", MIX_EP8 + " --steps 3 --warmup 2", 500),
                 run("ep8_hot_cf1125", DPO + " --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8"
                     " --ep-capacity 1.125 --ep-hot --steps 3 --warmup 2", 500),
                 run("ep8_bal_cf1125", DPO + " --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8"
                     " --ep-capacity 1.125 --steps 3 --warmup 2", 500)],
    # the new decode default at the GEN8 shape (prompt 1024 + 128) vs the round-5 rule (min 3)
    "r6-gen8-ab": [ab("gen8_loopmin", GEN8, {"new": {}, "min3": {"DLA_DECODE_LOOP_MIN": "3"}}, 2, 300),
                   ab("gen_rlhf_loopmin", "python -u tools/bench_generate.py --modes graph --prompt 512 --new 256",
                      {"new": {}, "min3": {"DLA_DECODE_LOOP_MIN": "3"}}, 1, 300)],
    # final-build DPO step: kernel categories + table, and one PMC pass over the library GEMMs and
    # the attention / SwiGLU kernels (MFMA busy, wave occupancy)
    "r6-final-prof": [prof("dpo", DPO + " --steps 2 --warmup 1", DPO_TABLES),
                      pmc("dpo_pmc", "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE",
                          "python3 bench.py --micro-pairs 4 --accum 1 --steps 1 --warmup 1",
                          "Cijk attn_fwd attn_bwd8 adamw swiglu_bwd_t logprob_bwd_t", 400, ["--by-grid"],
                          "Cijk|attn_fwd|attn_bwd8|adamw|swiglu_bwd_t|logprob_bwd_t")],
    # dense input gradients through the cached W^T (TN, refreshed every step) vs dY @ W (NN)
    "r6-dgrad-ab": [ab("dgrad_layout", DPO + " --steps 5 --warmup 2", {"tn": {"DLA_TRANSPOSED_DGRAD": "1"},
                                                                     "nn": {"DLA_TRANSPOSED_DGRAD": "0"}}, 2, 300)],
    # B = 8 decode gate|up kernel variants at the RLHF shape (round-6 build)
    "r6-glu-ab": [ab("glu", "python -u tools/bench_generate.py --modes graph --prompt 512 --new 256",
                     {"lds": {}, "il": {"DLA_DECODE_GLU_IL": "1"}, "ks": {"DLA_SKINNY_GLU": "ks"}}, 2, 300)],
    "r6-glu-ab2": [ab("glu_rlhf", "python -u tools/bench_generate.py --modes graph --prompt 512 --new 256",
                      {"lds": {}, "ks": {"DLA_SKINNY_GLU": "ks"}}, 3, 300),
                   ab("glu_gen8", GEN8, {"lds": {}, "ks": {"DLA_SKINNY_GLU": "ks"}}, 3, 300)],
    # PPO with the critic on its side stream in the stats pass and the update vs one stream
    "r6-ppo-ab": [pytest("tests/test_ppo_shape.py", 300),
                  ab("ppo_critic_stream2", "python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8",
                     {"side": {"DLA_PPO_CRITIC_STREAM": "1"}, "one": {"DLA_PPO_CRITIC_STREAM": "0"}}, 2, 500)],
    # B = 8 graph decode at the RLHF shape under a kernel trace (per-layer kernel costs)
    "r6-dec-prof": [prof("gen_rlhf", "python -u tools/bench_generate.py --modes graph --prompt 512 --new 256",
                         [("window", ["--by-grid", "--top", "30", "--per", "8192"])], 300)],
    # load-adaptive library rows for the single local expert (parallel.expert ADAPTIVE_MAIN)
    "r6-mixtral2": [pytest("tests/test_moe_gpu.py", 400),
                    run("ep8_hot", MIX_EP8 + " --ep-hot --steps 3 --warmup 2", 500),
                    run("ep8_bal", MIX_EP8 + " --steps 3 --warmup 2", 500),
                    run("ep8_hot_cf1125", DPO + " --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8"
                        " --ep-capacity 1.125 --ep-hot --steps 3 --warmup 2", 500),
                    run("ep8_hot_fp8", MIX_EP8 + " --ep-hot --fp8 --steps 3 --warmup 2", 500),
                    run("ep8_bal_fp8", MIX_EP8 + " --fp8 --steps 3 --warmup 2", 500)],
    # RLHF forced vs plain after the one-rank groups went back to the normal-priority RCCL stream
    "r6-rlhf3": [run("rlhf_plain0", "python -u tools/bench_rlhf.py --batch 8", 400),
                 run("rlhf_forced0", "python -u tools/bench_rlhf.py --batch 8 --force-pg", 400),
                 run("rlhf_plain1", "python -u tools/bench_rlhf.py --batch 8", 400),
                 run("rlhf_forced1", "python -u tools/bench_rlhf.py --batch 8 --force-pg", 400),
                 run("dpo_force_pg", DPO + " --force-pg --steps 5 --warmup 2", 300),
                 run("dpo_plain", DPO + " --steps 5 --warmup 2", 300)],
    # which part of the forced one-rank RCCL path slows the RLHF update (no comm kernels run)
    "r6-forced-probe": [ab("rlhf_forced_env", "python -u tools/bench_rlhf.py --batch 8 --force-pg",
                           {"base": {}, "lowprio": {"DLA_RCCL_HIGH_PRIORITY": "0"},
                            "no_ag_overlap": {"DLA_OVERLAP_AG": "0"},
                            "no_async_err": {"TORCH_NCCL_ASYNC_ERROR_HANDLING": "0"},
                            "pg_only": {"DLA_BENCH_ENGINE_PLAIN": "1"}}, 1, 400)],
    # the whole DPO step's launches in issue order (which GEMM runs where, at what cost in place)
    # and the GEMM probe's arms under a kernel trace (which library kernel each form picks)
    "r6-seq": [prof("dpo_seq", DPO + " --steps 2 --warmup 1", [("window", ["--window", "adamw", "--seq", "0:7000"])]),
               prof("gemm_probe", "python -u tools/gemm_m_probe.py --model llama3-8b --ms 8192 --resid",
                    [("window", ["--by-grid", "--top", "40"])], 300)],
    # ---- round 5
    # DPO step GEMMs: MFMA busy and effective clock per library GEMM shape (by grid)
    "dpo-gemm-pmc": [pmc("dpo_gemm", "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE",
                         "python3 bench.py --micro-pairs 4 --accum 1 --steps 1 --warmup 1",
                         "Cijk attn_fwd attn_bwd8 adamw swiglu_bwd_t", 400, ["--by-grid"],
                         "Cijk|attn_fwd|attn_bwd8|adamw|swiglu_bwd_t")],
    # long-context DPO on the final build (the shard one SP-group member runs)
    "longctx": [run("longctx_4k", DPO + " --seq-len 4096 --micro-pairs 1 --accum 4 --steps 3 --warmup 1", 400),
                run("longctx_8k", DPO + " --seq-len 8192 --micro-pairs 1 --accum 2 --steps 3 --warmup 1", 400),
                run("ref_fp8", DPO + " --steps 5 --warmup 2", 300, {"DLA_REF_FP8": "1"})],
    # B = 64 decode attention: key splits per sequence (DLA_DECODE_BLOCKS = target grid)
    "ab-b64-blocks": [ab("b64_blocks", GEN64, {"base": {}, "blk1024": {"DLA_DECODE_BLOCKS": "1024"},
                                               "blk2048": {"DLA_DECODE_BLOCKS": "2048"}}, 2, 300)],
    "force-pg": [
        pytest("tests/test_force_comm.py -m gpu", 400),
        prof("force_pg", DPO + " --force-pg --steps 2 --warmup 1",
             [("streams", ["--window", "adamw"])]),
        ab("force_pg_ab", DPO + " --steps 5 --warmup 2", {"plain": {}, "forced": {"DLA_FORCE_PG": "1"}}, 2, 300),
    ],
    "meshes": [
        run("tp8", L70 + " --tp-shape 8 --micro-pairs 2 --accum 8", 330),
        run("fsdp2tp4", L70 + " --zero 3 --fsdp-shape 2 --tp-shape 4 --micro-pairs 2 --accum 8", 360),
        run("fsdp8", L70 + " --zero 3 --fsdp-shape 8 --micro-pairs 1 --accum 16", 420),
        run("mixtral_ep4edp2", MIX_EP8.replace("--ep-shape 8", "--ep-shape 4 --edp-shape 2") + " --steps 3 --warmup 1", 400),
        run("mixtral_ep8", MIX_EP8 + " --steps 3 --warmup 1", 400),
    ],
    # ---- kernel tables and counters (round 4 passes 2/3/16/26/37)
    "dpo-profile": [prof("dpo", DPO + " --steps 2 --warmup 1", DPO_TABLES)],
    "rlhf-overlap": [
        ab("rlhf_overlap_ab", "python -u tools/bench_rlhf.py --batch 8 --force-pg --steps 3 --warmup 1",
           {"sync": {}, "overlap": {"DLA_BENCH_RLHF_OVERLAP": "1"}}, 1, 500),
        prof("rlhf_overlap", "python -u tools/bench_rlhf.py --batch 8 --force-pg --overlap --steps 2 --warmup 1",
             [("streams", ["--pairs", "4"])], 500),
    ],
    "ppo-profile": [prof("ppo", "python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8 --steps 1 --warmup 1",
                         [("breakdown", []), ("window", ["--by-grid", "--top", "40"])], 500)],
    "decode-profile": [prof("dec8", GEN8, DEC_TABLE, 300), prof("dec64", GEN64, DEC_TABLE, 300)],
    "decode-fp8-profile": [prof("dec8_fp8", GEN8 + " --weight-dtype fp8", DEC_TABLE, 300),
                           prof("dec8_bf16", GEN8, DEC_TABLE, 300)],
    "decode64-fp8-profile": [prof("dec64_fp8", GEN64 + " --weight-dtype fp8", DEC_TABLE, 300),
                             prof("dec64_bf16", GEN64, DEC_TABLE, 300)],
    "mixtral-profile": [prof("mixtral", MIX_EP8 + " --steps 2 --warmup 1",
                             [("breakdown", []), ("window", ["--window", "adamw", "--top", "45"])])],
    "attn-pmc": [pmc("attn_p1", ATTN_P1, "python3 tools/attn_bench.py --iters 3",
                     "attn_fwd attn_bwd8 attn_dq_reduce attn_dkv_reduce", 150),
                 pmc("attn_p2", ATTN_P2, "python3 tools/attn_bench.py --iters 3",
                     "attn_fwd attn_bwd8 attn_dq_reduce attn_dkv_reduce", 150)],
    "decode64-pmc": [pmc("dec64", "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
                         "SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE FETCH_SIZE",
                         "python3 tools/bench_generate.py --modes eager --new 4 --batch 64 --prompt 512",
                         "m64_gemm m64_reduce decode_attn_loop")],
    "tp-chunks": [run("tp_chunk_probe", "python -u tools/tp_chunk_probe.py", 300)],
    # ---- round-4 A/Bs whose knobs are still in the tree (results in README "Tried, measured")
    "ab-dq-bf16": [ab("dq_bf16", DPO + " --steps 4 --warmup 2", {"on": {"DLA_ATTN_DQ_BF16": "1"},
                                                                 "off": {"DLA_ATTN_DQ_BF16": "0"}}, 1, 400)],
    "ab-tn-wgrad-max": [ab("tn_max", DPO + " --steps 6 --warmup 2",
                           {"inf": {"DLA_TN_WGRAD_MAX": "4611686018427387904"},
                            "3e8": {"DLA_TN_WGRAD_MAX": "300000000"}}, 2, 400)],
    "ab-tn-wgrad-min": [ab("tn_min", MIX_EP8 + " --steps 3 --warmup 2",
                           {"1Mi": {"DLA_TN_WGRAD_MIN": "1048576"}, "0": {"DLA_TN_WGRAD_MIN": "0"}})],
    "ab-micro-shape": [ab("micro_4x4", DPO + " --micro-pairs 4 --accum 4 --steps 6 --warmup 2", {"4x4": {}}, 2, 400),
                       ab("micro_8x2", DPO + " --micro-pairs 8 --accum 2 --steps 6 --warmup 2", {"8x2": {}}, 2, 400)],
    "ab-mixtral-single-lib": [pytest("tests/test_moe_gpu.py -m gpu", 300),
                              ab("single_lib", MIX_EP8 + " --steps 3 --warmup 2",
                                 {"lib+route": {"DLA_MOE_SINGLE_LIB": "1", "DLA_EP_NATIVE_ROUTE": "1"},
                                  "lib": {"DLA_MOE_SINGLE_LIB": "1", "DLA_EP_NATIVE_ROUTE": "0"},
                                  "neither": {"DLA_MOE_SINGLE_LIB": "0", "DLA_EP_NATIVE_ROUTE": "0"}}, 1)],
    "mixtral-ep-degrees": [run(f"ep{ep}", MIX_EP8.replace("--ep-shape 8", f"--ep-shape {ep}") + " --steps 3 --warmup 2")
                           for ep in (4, 2)],
    "ab-decode-blocks": [ab("blocks", GEN8, {"base": {"DLA_DECODE_RING": "2"},
                                             "b64r3": {"DLA_DECODE_BLOCKS": "64", "DLA_DECODE_RING": "3"},
                                             "b128r3": {"DLA_DECODE_BLOCKS": "128", "DLA_DECODE_RING": "3"},
                                             "b96r3": {"DLA_DECODE_BLOCKS": "96", "DLA_DECODE_RING": "3"},
                                             "b64r2": {"DLA_DECODE_BLOCKS": "64", "DLA_DECODE_RING": "2"}}, 2, 300)],
    "ab-kv-head-major": [pytest("tests -m gpu"),
                         ab("khm_b64", GEN64, {"hm": {"DLA_KV_HEAD_MAJOR": "1"}, "tm": {"DLA_KV_HEAD_MAJOR": "0"}}, 2, 300),
                         ab("khm_b8", GEN8, {"hm": {"DLA_KV_HEAD_MAJOR": "1"}, "tm": {"DLA_KV_HEAD_MAJOR": "0"}}, 2, 300)],
}


class Runner:
    def __init__(self, out: str, dry: bool):
        self.out, self.dry = out, dry
        os.makedirs(out, exist_ok=True)

    def _call(self, cmd, timeout_s, log, env=None, cwd=ROOT):
        full = ["timeout", "-k", "10", str(timeout_s)] + (cmd if isinstance(cmd, list) else shlex.split(cmd))
        if self.dry:
            print("DRY", " ".join(f"{k}={v}" for k, v in (env or {}).items()), " ".join(full))
            return 0
        e = dict(os.environ, PYTHONUNBUFFERED="1", TMPDIR="/tmp", **(env or {}))
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        with open(log, "w") as fh:
            return subprocess.call(full, cwd=cwd, env=e, stdout=fh, stderr=subprocess.STDOUT)

    @staticmethod
    def _last(log):
        try:
            lines = [ln for ln in open(log, errors="replace").read().splitlines() if ln.strip()]
        except OSError:
            return ""
        return lines[-1][:400] if lines else ""

    def _check(self, rc, what, log):
        if rc != 0:
            print(f"FAILED {what} rc={rc}; tail of {log}:")
            try:
                print("\n".join(open(log, errors="replace").read().splitlines()[-30:]))
            except OSError:
                pass
            raise SystemExit(1)

    def step(self, s):
        k, t = s["kind"], s["timeout"]
        o = self.out
        if k == "pytest":
            log = f"{o}/pytest_{abs(hash(s['sel'])) % 10000}.log"
            cmd = f"python -u -m pytest {s['sel']} -x -q --timeout 200 --timeout-method thread"
            self._check(self._call(cmd, t, log), s["sel"], log)
            print(f"pytest {s['sel']}: {self._last(log)}")
        elif k == "smoke":
            log = f"{o}/smoke.log"
            cmd = ["python", "-u", "-c", "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')"]
            self._check(self._call(cmd, t, log), "smoke", log)
            print("smoke:", self._last(log))
        elif k == "run":
            log = f"{o}/{s['name']}.log"
            self._check(self._call(s["cmd"], t, log, s["env"]), s["name"], log)
            print(f"{s['name']}: {self._last(log)}")
        elif k == "ab":
            for r in range(s["rounds"]):
                for arm, env in s["arms"].items():
                    log = f"{o}/{s['name']}_{arm}.{r}.log"
                    self._check(self._call(s["cmd"], t, log, env), f"{s['name']}/{arm}", log)
                    print(f"{s['name']} arm={arm} r={r}: {self._last(log)}")
        elif k == "prof":
            d = f"/tmp/prof_{s['name']}"
            shutil.rmtree(d, ignore_errors=True)
            log = os.path.abspath(f"{o}/prof_{s['name']}.log")
            cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--"] \
                + shlex.split(s["cmd"].replace("python -u ", "python3 -u ").replace("python ", "python3 "))
            self._check(self._call(cmd, t, log, s["env"]), f"prof {s['name']}", log)
            if self.dry:
                return
            tr = (glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True) or [None])[0]
            if tr is None:
                self._check(1, f"prof {s['name']} (no kernel trace)", log)
            tools = {"window": "prof_window.py", "breakdown": "step_breakdown.py", "streams": "prof_streams.py"}
            kinds = [k for k, _ in s["summaries"]]
            for i, (kind, args) in enumerate(s["summaries"]):
                dup = kinds.count(kind) > 1 and kinds.index(kind) != i
                dst = f"{o}/{s['name']}_{kind}{i if dup else ''}.md"
                with open(dst, "w") as fh:
                    rc = subprocess.call([sys.executable, os.path.join(ROOT, "scripts", tools[kind]), tr, *args],
                                         stdout=fh, stderr=subprocess.STDOUT)
                self._check(rc, f"summary {dst}", dst)
                print(f"prof {s['name']}: {dst}")
            shutil.rmtree(d, ignore_errors=True)
        elif k == "pmc":
            d = f"/tmp/pmc_{s['name']}"
            shutil.rmtree(d, ignore_errors=True)
            log = os.path.abspath(f"{o}/pmc_{s['name']}.log")
            inc = ["--kernel-include-regex", s["include"]] if s.get("include") else []
            cmd = ["rocprofv3", "--pmc", *s["counters"].split(), *inc, "--output-format", "csv", "-d", d, "-o", "run",
                   "--", *shlex.split(s["cmd"])]
            full = ["timeout", "-s", "KILL", str(t)] + cmd
            if self.dry:
                print("DRY", " ".join(full))
                return
            with open(log, "w") as fh:
                rc = subprocess.call(full, cwd=ROOT, stdout=fh, stderr=subprocess.STDOUT,
                                     env=dict(os.environ, TMPDIR="/tmp"))
            self._check(rc, f"pmc {s['name']}", log)
            c = (glob.glob(f"{d}/**/*counter_collection.csv", recursive=True) or [None])[0]
            dst = f"{o}/{s['name']}_pmc.md"
            with open(dst, "w") as fh:
                rc = subprocess.call([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary_csv.py"), c,
                                      *s.get("summary_args", []), "-k", *s["kernels"].split()],
                                     stdout=fh, stderr=subprocess.STDOUT)
            self._check(rc, f"pmc summary {dst}", dst)
            shutil.rmtree(d, ignore_errors=True)
            print(f"pmc {s['name']}: {dst}")
        else:
            raise ValueError(k)




def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("name", nargs="?")
    ap.add_argument("--out", default=None)
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--dry", action="store_true", help="print the commands only")
    a = ap.parse_args(argv)
    if a.list or not a.name:
        for n, steps in PASSES.items():
            print(f"{n:24s} {len(steps)} step(s): " + ", ".join(s.get("name", s["kind"]) for s in steps))
        return 0
    if a.name not in PASSES:
        raise SystemExit(f"unknown pass {a.name!r} (--list)")
    out = a.out or os.path.join(ROOT, "gpurun_out", a.name)
    r = Runner(out, a.dry)
    stop = threading.Event()

    def beat():
        while not stop.wait(30):
            with open(os.path.join(out, "heartbeat"), "w") as fh:
                fh.write(time.ctime())

    threading.Thread(target=beat, daemon=True).start()
    try:
        for s in PASSES[a.name]:
            r.step(s)
    finally:
        stop.set()
    print("ALL_DONE")
    return 0


if __name__ == "__main__":
    sys.exit(main())
