/*
 * f5h.h — C ABI of the MI355X (gfx950) CFM sampling engine.
 *
 * The engine replaces the hot path of the reference:
 *   CFM.sample()            /root/reference/src/f5_tts/model/cfm.py:83-229   (Euler ODE + CFG loop)
 *   DiT.forward()           /root/reference/src/f5_tts/model/backbones/dit.py:319-370
 *   UNetT.forward()         /root/reference/src/f5_tts/model/backbones/unett.py:244-307
 * behind the reference's own Python surface (`model_obj.sample(...)`, called from
 * infer/utils_infer.py:497-504, eval/eval_infer_batch.py:190-200, runtime/.../benchmark.py:415-423).
 *
 * Plain C types only: pointers, sizes, ints. No torch types cross this boundary.
 * Every entry point returns 0 on success, a negative f5h_status otherwise; the
 * message is available from f5h_last_error() (thread-local).
 *
 * Ownership: the engine owns its packed device weights and is immutable after
 * f5h_engine_create (shareable between host threads). The caller owns every I/O
 * buffer and the workspace, so concurrent calls on different workspaces are
 * re-entrant (this replaces the reference's thread-local text cache, dit.py:237-262).
 * All work is enqueued on the caller's hipStream_t (passed as void*).
 */
#ifndef F5H_H
#define F5H_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum f5h_status {
  F5H_OK = 0,
  F5H_EINVAL = -1,   /* bad argument / shape */
  F5H_EHIP = -2,     /* HIP runtime error */
  F5H_ENOWEIGHT = -3,/* missing or mis-shaped weight */
  F5H_ENOMEM = -4,   /* workspace too small */
};

enum f5h_backbone { F5H_DIT = 0, F5H_UNETT = 1 };
/* Operand dtype of the GEMM / attention / conv MFMAs. Accumulation, norm and softmax statistics and
 * the ODE state are fp32 in every mode; the residual stream is fp32 in the fp32 mode and, in the 16-bit
 * modes, kept in the operand dtype on both backbones (DiT and UNetT), as the reference keeps it in the
 * parameter dtype.
 *   F5H_FP32: parity mode (exact-f32 MFMA, VALU attention), the <=1e-3 contract;
 *   F5H_BF16: bf16 operands (the BASELINE configs' dtype);
 *   F5H_FP16: fp16 operands = the reference's default GPU dtype (load_checkpoint casts to fp16 on
 *             any GPU with compute capability >= 7, utils_infer.py:190-199); same MFMA rate as bf16. */
enum f5h_compute { F5H_FP32 = 0, F5H_BF16 = 1, F5H_FP16 = 2 };

/* Architecture: mirrors DiT.__init__ (dit.py:171-192) / UNetT.__init__ (unett.py:108-129)
 * and the Hydra arch block (configs/F5TTS_v1_Base.yaml:24-37). */
typedef struct f5h_arch {
  int32_t backbone;          /* f5h_backbone */
  int32_t dim;               /* model width d (multiple of 64) */
  int32_t depth;             /* blocks */
  int32_t heads;             /* attention heads */
  int32_t dim_head;          /* must be 64 */
  int32_t ff_dim;            /* int(dim * ff_mult) */
  int32_t text_dim;          /* text embedding width (DiT: 512; UNetT: mel_dim) */
  int32_t text_num_embeds;   /* vocab size (embedding has text_num_embeds+1 rows) */
  int32_t mel_dim;           /* 100 */
  int32_t conv_layers;       /* ConvNeXtV2 text blocks */
  int32_t text_mask_padding; /* 0/1 */
  int32_t pe_attn_head;      /* 0 = rope on all heads, k>0 = first k heads (modules.py:503-506) */
  int32_t attn_mask_enabled; /* 0/1: key-padding mask in attention (modules.py:512-516) */
  int32_t compute;           /* f5h_compute: FP32 parity mode, BF16 or FP16 MFMA mode */
} f5h_arch;

/* One named parameter, host memory, float32, C-contiguous, with the reference's
 * state-dict name minus the `transformer.` prefix (e.g. "transformer_blocks.3.attn.to_q.weight"). */
typedef struct f5h_weight {
  const char* name;
  const float* data;
  int64_t numel;
} f5h_weight;

/* Element type of a weight view. */
enum f5h_dtype { F5H_DT_F32 = 0, F5H_DT_BF16 = 1, F5H_DT_F16 = 2 };

/* One named parameter in its own dtype and placement: host memory, or device memory
 * of the engine's device (e.g. a torch parameter's data_ptr() after model.to(dtype).to(device), as
 * load_checkpoint leaves it, utils_infer.py:190-232). C-contiguous, state-dict name as f5h_weight. */
typedef struct f5h_tensor_view {
  const char* name;
  const void* data;
  int32_t dtype;             /* f5h_dtype */
  int32_t on_device;         /* 0: host memory; 1: device memory of `device` */
  int64_t numel;
} f5h_tensor_view;

typedef struct f5h_engine f5h_engine;

/* Replaces: model construction + load_checkpoint (utils_infer.py:190-276): packs the
 * weights into the engine's device layout (bf16/fp16/fp32 GEMM panels, conv taps, the
 * concatenated AdaLN matrix). Host views are staged to the device in their own dtype; every
 * panel is packed on the device (no host fp32 copy of the model). Blocks until packing is complete;
 * the views may be released afterwards. Device views are read on the engine's own non-blocking stream,
 * ordered behind the null stream (hence behind work queued on blocking streams): the caller must have
 * completed any write to them still queued on a non-blocking stream (e.g. a torch side stream). */
int f5h_engine_create_views(const f5h_arch* arch, const f5h_tensor_view* weights, int32_t n_weights,
                            int32_t device, f5h_engine** out);
/* The same from fp32 host arrays (f5h_weight). */
int f5h_engine_create(const f5h_arch* arch, const f5h_weight* weights, int32_t n_weights,
                      int32_t device, f5h_engine** out);
/* Returns at once. The engine's device resources are released on a background thread once the
 * engine's own work has completed (per stream, an event recorded after each call; the events after its
 * graph replays): no device-wide synchronisation, so dropping an engine never waits for other streams.
 * The same holds for f5h_vocos_destroy and f5h_mel_destroy. */
void f5h_engine_destroy(f5h_engine* eng);
/* Releases still queued or running (engines, Vocos and log-mel objects destroyed above); wait != 0
 * first blocks until every one of them has completed (also run at process exit). The objects' device
 * memory comes from a stream-ordered pool per device that keeps released memory for reuse (so neither
 * creation nor release synchronises the device); wait == 2 then also returns the pool's unused memory
 * to the system, which waits for the device. */
int f5h_release_pending(int32_t wait);

/* Arguments of one CFM.sample call after the host preamble of cfm.py:105-158 and
 * the noise/time-grid recipe of cfm.py:196-216. All pointers are DEVICE pointers
 * except t_grid (host). Shapes: B utterances, N = max duration (padded frames),
 * nt text tokens. */
typedef struct f5h_sample_args {
  int32_t B, N, nt, nfe;
  const float* cond;         /* [B,N,mel] padded cond mel (cfm.py:148) */
  const uint8_t* cond_mask;  /* [B,N] 1 = keep cond (lens_to_mask(lens) & edit_mask, cfm.py:128-130) */
  const int64_t* text;       /* [B,nt] token ids, -1 = pad (utils.py:99-106) */
  const int32_t* duration;   /* [B] per-utterance total frames (cfm.py:135-139) */
  const float* y0;           /* [B,N,mel] initial noise, zero-padded (cfm.py:196-201) */
  const float* t_grid;       /* HOST [nfe+1] time grid, EPSS/linspace + sway (cfm.py:211-216) */
  float cfg_strength;        /* < 1e-5 disables the packed uncond branch (cfm.py:167) */
  int32_t use_batch_mask;    /* 1 when B>1 (cfm.py:155-158) */
  float* out;                /* [B,N,mel] result: where(cond_mask, cond, y_final) (cfm.py:223) */
  float* trajectory;         /* [nfe+1,B,N,mel] or NULL (odeint output, cfm.py:218) */
} f5h_sample_args;

/* Bytes of workspace f5h_sample needs for a call of this shape. */
size_t f5h_workspace_size(const f5h_engine* eng, int32_t B, int32_t N, int32_t nt, int32_t nfe,
                          int32_t use_cfg);

/* Replaces CFM.sample's ODE loop (cfm.py:160-223): text embedding once, then nfe Euler
 * steps each running one packed cond/uncond backbone forward, CFG combine and the update,
 * then the final cond overwrite. Everything enqueued on `stream` (a hipStream_t). */
int f5h_sample(f5h_engine* eng, void* stream, const f5h_sample_args* args, void* workspace,
               size_t workspace_bytes);

/* One backbone forward: the backbone plugin contract DiT.forward / UNetT.forward
 * (dit.py:319-370, unett.py:244-307) with a scalar time t.
 *   cfg_infer = 1: the packed cond/uncond forward CFM.sample uses (cfm.py:181-191): pred [2B,N,mel],
 *                  conditional rows then unconditional rows (drop flags ignored);
 *   cfg_infer = 0: one branch (cfm.py:167-178), pred [B,N,mel], honouring drop_audio_cond (cond -> 0,
 *                  InputEmbedding, dit.py:155-156) and drop_text (all-filler text ids, dit.py:106-107).
 * x [B,N,mel]; step_cond = where(cond_mask, cond, 0) is formed from cond/cond_mask. Per-sample time
 * values are served by the caller in groups of equal t (sequences are independent at equal N). */
typedef struct f5h_forward_args {
  int32_t B, N, nt;
  const float* x;
  const float* cond;
  const uint8_t* cond_mask;
  const int64_t* text;
  const int32_t* duration;
  float t;
  int32_t use_batch_mask;
  float* pred;               /* [2B,N,mel] (cfg_infer) or [B,N,mel] */
  int32_t cfg_infer;
  int32_t drop_audio_cond;
  int32_t drop_text;
  const float* t_dev;        /* DEVICE fp32 scalar time (read on the stream, no host sync), or NULL: use t */
  /* The reference's text cache (dit.py:294-317: with cache=True the first forward of a sample()
   * computes text_cond/text_uncond, later forwards reuse them until clear_cache()):
   *   0: compute the text embedding (both branches) for this call only;
   *   1: compute it and keep it in `workspace` for later calls;
   *   2: reuse the one kept in `workspace` (same B, N, nt; the text and durations of the keeping call).
   * With 1 or 2 the backbone step runs as a captured graph keyed by the workspace (graph mode). */
  int32_t text_cache;
} f5h_forward_args;
int f5h_forward(f5h_engine* eng, void* stream, const f5h_forward_args* args, void* workspace,
                size_t workspace_bytes);

/* Kernel probe: when enabled, every launch of kernel class `kclass` is timed on the device wall
 * clock (s_memrealtime): GEMM and attention kernels stamp their own entry/exit, the other classes
 * get a stamp kernel on each side (no HIP events, so it also times graph replays; every 4th NFE
 * step is sampled). f5h_probe_read returns (sampled launches, total ms). Enabling resets the slots
 * and synchronises the device. Classes: 0 = FFN1 GEMM, 1 = attention, 2 = QKV GEMM, 3 = FFN2 GEMM,
 * 4 = conv, 5 = attention output-projection GEMM, 6 = pre-FFN norm (LayerNorm+modulate / RMSNorm), 7 = the phase
 * chain launch (f5h_set_chain; its timeline row per workgroup: entry, rows acquired, results stored, exit). While
 * one of the classes 0, 2, 3, 5, 6 is probed the chain is off (those launches are timed one by one). */
int f5h_probe_enable(f5h_engine* eng, int32_t kclass, int32_t enable);
int f5h_probe_read(f5h_engine* eng, int64_t* launches, double* total_ms);
/* Per-workgroup timeline of the probed class's first launch in the first probed step (GEMM and
 * attention kernels): stamps[4*w + {0 entry, 1 main loop entered, 2 main loop done, 3 exit}] in ticks of
 * the device wall clock (tick_khz); n_wg = workgroups recorded (at most max_wg, at most 8192). */
int f5h_probe_timeline(f5h_engine* eng, uint64_t* stamps, int32_t max_wg, int32_t* n_wg, double* tick_khz);

/* NFE-step graph (the CFM.sample ODE loop, cfm.py:218 -> torchdiffeq Euler): with mode 1 (default;
 * env F5H_GRAPH=0 selects 0 at engine creation) f5h_sample captures one NFE step -- table-row
 * copy, backbone forward, CFG combine + Euler update, device step counter -- into a hipGraph on
 * first use and replays it nfe times; mode 0 launches the same sequence eagerly. The step touches
 * only workspace buffers, so the graph is keyed by (workspace, B, N, nfe, cfg, mask, probe,
 * kernel epoch); the caller's out/trajectory pointers are staged into the workspace per call.
 * The call prologue (time/AdaLN tables, text embedding, hoisted input projection) is captured as
 * a graph of its own only when its shape repeats (the first call of a shape runs it eagerly; env
 * F5H_PROLOGUE_GRAPH=0: always eager). Results are bitwise identical in every mode.
 * f5h_graph_stats: captures so far and graph replays so far (prologue and step graphs together),
 * graphs cached (LRU of 16 over both kinds). An evicted graph is destroyed later, without any host
 * wait, once the events recorded after its replays have completed and no caller holds it. */
int f5h_set_graph_mode(f5h_engine* eng, int32_t mode);
/* Launch chains of the captured step: 2 captures the conditional and the unconditional CFG branch as
 * two parallel chains (fork/join by events), so kernel boundaries of one branch overlap work of the
 * other; 1 = one chain over the packed batch; 0 = automatic (the default: currently one chain, measured
 * faster at C2, C3 and C5 and 0.7 % slower at C4; env F5H_SPLIT_CFG=0/1/2 = never/always/auto at engine
 * creation). Results are bitwise identical. */
int f5h_set_cfg_streams(f5h_engine* eng, int32_t n);
int f5h_graph_stats(f5h_engine* eng, int64_t* captures, int64_t* replays, int32_t* cached);
/* Host milliseconds the engine's newest f5h_sample call spent, by phase (a call that blocks its host thread
 * shows where): ms[0] whole call, [1] prologue (enqueue, or graph stage + launch), [2] waiting for the graph
 * cache lock, [3] destroying evicted graphs, [4] capturing, [5] instantiating, [6] launching the step graphs /
 * steps, [7] final kernel + fault-word copy. Writes min(n, 8) values, zeros past 8. */
int f5h_last_call_host_ms(f5h_engine* eng, double* ms, int32_t n);
/* Batch path (use_batch_mask): pad query rows' attention output is zeroed after to_out
 * (modules.py:551-553), so attention query blocks past a sequence's length exit at entry and out-proj row
 * tiles of padding only skip their work (the rows keep their residual, as masked rows of a computed tile
 * do). 1 (default; env F5H_NO_PAD_SKIP=1 at creation: 0) or 0 to compute every block. Bitwise identical. */
int f5h_set_pad_skip(f5h_engine* eng, int32_t enable);
/* 16-bit DiT path without row masks: run each layer's out-proj, LayerNorm, FFN1, FFN2 and the next layer's
 * LayerNorm + QKV (modules.py:743-757) as ONE launch whose phases hand 64-row groups to each other through
 * arrival counters (chain.hip, DESIGN.md §3 'Phase chain'), instead of six launches. 0 (default) or 1 (env
 * F5H_CHAIN=1 at creation: 1). Bitwise identical results; slower than the separate launches at C2 (58.4 vs
 * 51.1 ms), hence off. */
int f5h_set_chain(f5h_engine* eng, int32_t enable);
/* LayerNorm fold (DESIGN.md §3 'LayerNorm fold'): on the 16-bit DiT path without row masks, the AdaLN LayerNorm +
 * modulate between a residual GEMM and its consumer (modules.py:325,753: out-proj -> FFN1, FFN2 -> the next QKV)
 * runs inside those two GEMMs instead of as a launch of its own: the producer also writes h (1 + scale) and per-row
 * (mean, M2) partials of h, the consumer normalises its accumulators, rstd (acc - mean u) + v with per-step vectors
 * u = (1 + scale) W^T, v = shift W^T computed once per call. Not bitwise the separate launches (the statistics and
 * the rounding point move): within the reduced-precision envelopes (tests/test_gpu_envelope.py). 1 (default) or 0
 * (env F5H_LNFOLD=0 at creation: 0). The same switch covers the UNetT RMSNorm fold (default 0 on UNetT engines,
 * F5H_LNFOLD=1: on; unett.py:300-301, x_transformers
 * RMSNorm): every FFN-norm and the attention-norms of the first half's layers 1.., on masked batches too; the
 * producers write per-row sums of squares, the consumers read the residual stream with W diag(g) built once per
 * engine. f5h_ln_fold_stats: *supported = 1 when the engine can fold (16-bit DiT with dim and ff_dim multiples of
 * 64, or 16-bit UNetT with dim a multiple of 64; dim <= 1024), *passes = backbone passes enqueued with a fold. */
int f5h_set_ln_fold(f5h_engine* eng, int32_t enable);
int f5h_ln_fold_stats(f5h_engine* eng, int32_t* supported, int64_t* passes);
/* Failure of the chain (never expected): a chain wait that gives up (a bounded spin of ~0.3 s) sets the
 * ENGINE's fault word; that call's `out` (f5h_sample) / `pred` (f5h_forward) is then all NaN, and the engine's
 * next f5h_sample / f5h_forward fails with F5H_EHIP (message in f5h_last_error), clears the word and turns the
 * chain off for the engine. Concurrency: a call that would chain while a chained call from another stream of
 * the same device is still enqueued or running takes the separate launches (two chain launches in flight starve
 * each other, DESIGN.md §3 'Phase chain'); results are bitwise the same either way.
 * Test hook: *launches = chain launches this engine has enqueued (eager launches and graph captures);
 * *fault = the engine's fault word (1: a wait gave up since it was last cleared; NOT cleared here: the next call
 * reports it); *refused = chained calls of this process sent to the separate launches by the concurrency rule.
 * Synchronous; call after the engine's work has completed. Any pointer may be NULL. */
int f5h_chain_stats(f5h_engine* eng, int64_t* launches, int32_t* fault, int64_t* refused);
/* Test hook: polls before a chain wait gives up (limit >= 0; 0 = at the first poll that finds its rows not yet
 * produced), -1 restores the default (~0.3 s). Applies to launches and graph captures made afterwards. */
int f5h_chain_debug_spin_limit(int64_t limit);

/* Op-level entry points (parity tests / microbenchmarks). Device pointers, row-major. */
/* C[M,N] = A[M,K] . W[N,K]^T + bias  (fp32 in/out; compute = F5H_FP32 or F5H_BF16 operands) */
int f5h_op_linear(void* stream, int32_t compute, int32_t M, int32_t N, int32_t K, const float* A,
                  const float* W, const float* bias, float* C, void* workspace, size_t workspace_bytes);
/* O[S,N,H*64] = softmax(Q K^T / 8 [+key mask]) V with Q,K,V [S,H,N,64] fp32;
 * kv_len: [S] valid keys per sequence or NULL. q_prescaled != 0: Q already carries
 * scale * log2(e) (the engine's layout: scores in log2 units). */
int f5h_op_attention(void* stream, int32_t compute, int32_t S, int32_t H, int32_t N, const float* Q,
                     const float* K, const float* V, const int32_t* kv_len, int32_t q_prescaled, float* O,
                     void* workspace, size_t workspace_bytes);

/* Tuning/test hook: pin the 16-bit GEMM tile configuration for all later launches in this
 * process (0, 1, 5, 11, 12, 13), or -1 to restore the automatic per-shape choice. */
int f5h_gemm_force_config(int32_t cfg);
/* Test hook: on != 0 makes every later 16-bit attention launch of this process rerun each workgroup's key
 * loop in its lazy-running-max form (the path a row takes when a score runs far above its first tile's max;
 * attention.hip), 0 restores the default. Results agree to rounding (tests/test_gpu_parity.py). */
int f5h_attn_force_safe(int32_t on);
/* Test hook (host only, no device needed): the batch path's pad-row skip test of a GEMM row tile
 * (modules.py:551-553): 1 if rows [m0, m0 + BM) of an M-row operand hold a live row, where sequence s owns
 * rows [s*live_seq, (s+1)*live_seq) and its first live_len[s] rows are live; 0 if every row is padding.
 * The device kernels run the same function (kernels.h tile_live_rows). */
int f5h_debug_tile_live(const int32_t* live_len, int32_t live_seq, int32_t M, int32_t m0, int32_t BM);

/* ---------------------------------------------------------------------------------------
 * Vocos decoder (mel -> waveform), SURVEY §8(f1): the step after the CFM path, replacing
 * `vocoder.decode(mel)` (infer/utils_infer.py:510-511; runtime/triton_trtllm/benchmark.py:435)
 * of the vocos package's mel-24khz model (Vocos.decode = backbone + ISTFTHead). Weights by the
 * vocos state-dict names ("backbone.embed.weight", "backbone.convnext.{i}.pwconv1.weight",
 * "head.out.weight", ...), fp32 host arrays. compute: F5H_BF16 runs the backbone GEMMs on bf16
 * MFMA; the head and the inverse STFT always run in fp32. */
typedef struct f5h_vocos_arch {
  int32_t input_channels;    /* 100 mel bins */
  int32_t dim;               /* 512 */
  int32_t intermediate_dim;  /* 1536 */
  int32_t num_layers;        /* 8 */
  int32_t n_fft;             /* 1024 (win_length = n_fft, hann, center padding) */
  int32_t hop_length;        /* 256 */
  int32_t compute;           /* f5h_compute */
} f5h_vocos_arch;
typedef struct f5h_vocos f5h_vocos;

int f5h_vocos_create(const f5h_vocos_arch* arch, const f5h_weight* weights, int32_t n_weights, int32_t device,
                     f5h_vocos** out);
void f5h_vocos_destroy(f5h_vocos* v);
size_t f5h_vocos_workspace_size(const f5h_vocos* v, int32_t B, int32_t T);
/* mel [B][input_channels][T] fp32 (vocos' channel-first layout) -> audio [B][(T-1)*hop] fp32
 * (torch.istft center=True length). Device pointers; work enqueued on `stream`. */
int f5h_vocos_decode(f5h_vocos* v, void* stream, int32_t B, int32_t T, const float* mel, float* audio,
                     void* workspace, size_t workspace_bytes);

/* ---------------------------------------------------------------------------------------
 * Log-mel front end (wav -> mel), SURVEY §8(f2): replaces get_vocos_mel_spectrogram
 * (model/modules.py:80-109; torchaudio MelSpectrogram power 1, center/reflect, periodic Hann,
 * htk filterbank without norm, f_max = sr/2; then clamp(1e-5).log()), which CFM.sample applies
 * to raw-audio conditioning (cfm.py:106-108). fp32 throughout (DFT and filterbank on fp32 MFMA). */
typedef struct f5h_mel_arch {
  int32_t n_fft;        /* 1024 (= win_length) */
  int32_t hop_length;   /* 256 */
  int32_t n_mels;       /* 100 */
  int32_t sample_rate;  /* 24000 */
} f5h_mel_arch;
typedef struct f5h_mel f5h_mel;

int f5h_mel_create(const f5h_mel_arch* arch, int32_t device, f5h_mel** out);
void f5h_mel_destroy(f5h_mel* m);
/* frames T = 1 + L / hop (torch.stft center=True); L must exceed n_fft/2 (reflect padding) */
size_t f5h_mel_workspace_size(const f5h_mel* m, int32_t B, int32_t L);
/* wav [B][L] fp32 -> mel [B][n_mels][T] fp32 (device pointers, enqueued on `stream`) */
int f5h_mel_forward(f5h_mel* m, void* stream, int32_t B, int32_t L, const float* wav, float* mel, void* workspace,
                    size_t workspace_bytes);

const char* f5h_last_error(void);
const char* f5h_version(void);

#ifdef __cplusplus
}
#endif
#endif /* F5H_H */
