/*
 * zipvoice_hip.h — C ABI of the MI355X-native ZipVoice inference engine
 * (libzipvoice_hip.so, gfx950).
 *
 * Plain pointers and sizes only.  Every tensor argument is a DEVICE pointer
 * (caller-owned, row-major, contiguous) unless the parameter name says host_.
 * All work is enqueued on `stream` (a hipStream_t, NULL = default stream); no
 * call synchronises the host except zv_finalize (weight upload).
 * Return value: 0 on success, nonzero on error; zv_last_error() then returns
 * a thread-local message (the Python layer raises it as RuntimeError /
 * ValueError, mirroring the reference's exceptions).
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repository winlaic/ZipVoice):
 *   zv_create / zv_set_weight / zv_finalize
 *       ZipVoice*.__init__ + load_checkpoint(strict=True)
 *       (zipvoice/models/zipvoice.py:38-133, zipvoice/utils/checkpoint.py:108-146,
 *        zipvoice/bin/infer_zipvoice.py:549-566)
 *   zv_fm_decoder      ZipVoice.forward_fm_decoder (zipvoice/models/zipvoice.py:135-185)
 *                      == TTSZipformer.forward (zipvoice/models/modules/zipformer.py:242-293)
 *   zv_velocity        DiffusionModel.forward / DistillDiffusionModel.forward
 *                      (zipvoice/models/modules/solver.py:40-165)
 *   zv_euler_sample    EulerSolver.sample (zipvoice/models/modules/solver.py:182-240)
 *   zv_text_encode     ZipVoice.forward_text_embed (zipvoice/models/zipvoice.py:187-212,
 *                      ZipVoiceDialog override zipvoice/models/zipvoice_dialog.py:127-159)
 *   zv_text_condition  ZipVoice.forward_text_condition (zipvoice/models/zipvoice.py:214-251)
 *   zv_speech_condition  speech-condition padding in ZipVoice.sample (zipvoice.py:441-451)
 *   Reference per-step ONNX operator with the same contract as zv_velocity:
 *       fm_decoder.onnx (zipvoice/bin/onnx_export.py:157-204)
 *   zv_vocoder_*       the vocoder the reference loads and calls after sampling:
 *                      get_vocoder (zipvoice/bin/infer_zipvoice.py:249-273) ->
 *                      Vocos.from_hparams + load_state_dict, and
 *                      `vocoder.decode(pred_features).squeeze(1).clamp(-1, 1)` with the
 *                      feature post-processing of infer_zipvoice.py:374-378
 *                      (third-party vocos 0.1.0: Vocos.decode = VocosBackbone + ISTFTHead)
 *   zv_fbank_*         VocosFbank.extract (zipvoice/utils/feature.py:36-120) and
 *                      BigVGANFbank.extract (:133-204, _bigvgan_mel_feature.py:42-111): the prompt
 *                      log-mel front end feeding prompt_features (infer_zipvoice.py:328-337)
 */
#ifndef ZIPVOICE_HIP_H
#define ZIPVOICE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct zv_engine* zv_handle;

enum zv_variant { ZV_ZIPVOICE = 0, ZV_DISTILL = 1, ZV_DIALOG = 2, ZV_DIALOG_STEREO = 3 };
/* ZV_FP32: fp32-accurate mode (GEMMs as split products hi*hi + hi*lo + lo*hi of 16-bit
 *          operands, fp32 everything else);
 * ZV_BF16: 16-bit MFMA operands, fp32 accumulation / residual stream / softmax;
 * ZV_MIXED: ZV_BF16 for the decoder layers, the split products for the decoder's input /
 *          output projections, the layers' attention-score projections and the whole text
 *          encoder (the cheap linears that carry most of the 16-bit rounding error into the
 *          output).
 * The 16-bit operand format is the library's: bf16 in libzipvoice_hip.so, IEEE fp16 in
 * libzipvoice_hip_f16.so (same entry points, built from the same sources with
 * -DZV_OPERAND_F16).  ZV_MIXED in the fp16 library is the parity-grade fast mode.
 * ZV_FP8: ZV_BF16 with the decoder layers' feed-forward, convolution-module and
 *          NonlinAttention output linears on block-scaled MX-fp8 MFMA (e4m3 weights and
 *          activations, one power-of-two scale per 32 K elements; bf16 library only).  The
 *          BASELINE C5 "fp8 MFMA weights" mode, with its own tolerance. */
enum zv_precision { ZV_FP32 = 0, ZV_BF16 = 1, ZV_MIXED = 2, ZV_FP8 = 3 };

#define ZV_MAX_STACKS 8

/* Mirrors the "model" block of model.json (egs/zipvoice/conf/zipvoice_base.json:2-25). */
typedef struct {
  int variant;                 /* zv_variant */
  int precision;               /* zv_precision */
  int feat_dim;                /* 100 */
  int num_stacks;              /* len(fm_decoder_downsampling_factor) */
  int downsampling_factor[ZV_MAX_STACKS];
  int num_layers[ZV_MAX_STACKS];
  int cnn_module_kernel[ZV_MAX_STACKS];
  int fm_decoder_dim, fm_decoder_feedforward_dim, fm_decoder_num_heads;
  int text_encoder_num_layers, text_encoder_feedforward_dim, text_encoder_cnn_module_kernel;
  int text_encoder_num_heads, text_encoder_dim;
  int time_embed_dim, text_embed_dim;
  int query_head_dim, value_head_dim, pos_head_dim, pos_dim;
  int vocab_size, pad_id, spk_a_id, spk_b_id;
} zv_config;

const char* zv_last_error(void);
const char* zv_version(void);

zv_handle zv_create(const zv_config* cfg);
void zv_destroy(zv_handle h);

/* Stage one state-dict tensor (host fp32, reference key name, e.g.
 * "fm_decoder.encoders.1.encoder.layers.0.feed_forward2.in_proj.weight"). */
int zv_set_weight(zv_handle h, const char* name, const float* host_data, int64_t numel);
/* Check that every tensor of the config's state dict was staged (strict=True),
 * convert/pad to the device layout and upload.  Synchronous. */
int zv_finalize(zv_handle h);
/* Pre-size the decoder workspace for guided calls of up to max_batch utterances of
 * max_frames frames (runs one uncaptured guided velocity on zeros and synchronises).
 * Optional: forward calls grow it on demand, which synchronises; after a reservation
 * no call up to that shape allocates device memory. */
int zv_reserve(zv_handle h, int max_batch, int max_frames);
/* Total bytes of device memory held (weights + workspace). */
int64_t zv_device_bytes(zv_handle h);

/* Launch profiler (process-wide): when enabled, every GEMM / attention launch is
 * bracketed by HIP events on its stream.  zv_profile(0/1) also clears the log
 * (2 = on, with GEMM records keyed by shape);
 * zv_profile_report writes a JSON object {kernel: {launches, flops, bytes, ms}}
 * (synchronises on the recorded events). */
int zv_profile(int enable);
int zv_profile_report(char* buf, int buflen);

/* Number of host-blocking HIP runtime calls the library has issued since load (process-wide:
 * allocations, frees, synchronous copies / memsets, device / stream / event synchronisation,
 * stream / event / graph creation and destruction).  A warm zv_euler_sample /
 * zv_vocoder_decode at an already-seen shape adds none: the per-rank step never waits on the
 * GPU inside the Euler loop (no reference counterpart: the reference's solver loop,
 * zipvoice/models/modules/solver.py:213-240, runs eagerly on the caller's stream). */
int64_t zv_host_block_count(void);

/* Exact-path counters of the second-generation attention consumers of the bf16 / fp8 engines
 * (csrc/zv_flash2.inc).  Those kernels take p = 2^s without subtracting a row maximum; a
 * SelfAttention wave or NonlinAttention block whose range check fails redoes its queries with the
 * maximum subtracted (the reference's softmax, zipformer.py:1257-1306).  host_counts[0]: runs with
 * a query denominator under 2^-60, [1]: over 2^100 or a non-finite accumulator, [2]: every run
 * (including those forced by ZV_ATTN2_EXACT=1, test infrastructure).  Synchronises the device;
 * reset = 1 zeroes the counters.  No reference counterpart (the reference materialises softmax). */
int zv_attn_fallbacks(zv_handle h, int reset, int64_t* host_counts);

/* The second-generation attention consumers alone, on host arrays (test infrastructure: pins
 * csrc/zv_flash2.inc against a float64 softmax in tests/test_gpu_attn2.py).  Inputs are rounded to
 * the operand format as the engine's producers round them.  qkp (B, L, 2*32*H + 4*H) fp32 rows
 * [q | k | p] in base-2 units (the engine folds log2(e) into the k / p weights); P (2L-1, 4*H) the
 * positional projection (base 2); key_pad (B, L) 1 = padded, or NULL (masked_fill(-1000) of
 * zipformer.py:1281-1289 in base 2).  kernel 0 = SelfAttention (zipformer.py:1359-1396): v (B, L,
 * H*nv), nv <= 12, out (B, L, H*nv); kernel 1 = NonlinAttention (zipformer.py:1499-1544, head 0):
 * v, y, out (B, L, nv), out = y * (W0 . v).  form 0 = the engine's choice for L (SelfAttention 1 / 2:
 * register-fed with 2 / 3 query tiles per wave, 3 / 4 / 5: LDS-ring with 2 / 3 / 4; NonlinAttention
 * 1 / 2: 4 / 8 query tiles per block).  force_exact = 1 sends every wave / block through the exact
 * path; counts (or NULL) receives the three zv_attn_fallbacks counters of this launch.  Operands
 * are the library's (bf16; fp16 in libzipvoice_hip_f16.so, whose kernels take p = 2^(s - o) with a
 * per-query offset o); synchronous. */
int zv_attn2_check(int kernel, int form, int B, int L, int H, int nv, const float* qkp, const float* P,
                   const uint8_t* key_pad, const float* v, const float* y, int force_exact, float* out,
                   int64_t* counts);

/* GEMM microbenchmark (random bf16 operands): average ms per launch of tile
 * variant `variant` (+100: one tile per block instead of the persistent grid) for
 * C(M,N) = A(M,K) W(N,K)^T with out_mode 0 = fp32 C, 1 = bf16 C, 2 = residual
 * (C += ..., fp32, plus a bf16 copy), 3 = SwooshL -> bf16. */
int zv_bench_gemm(int M, int N, int K, int variant, int iters, int out_mode, float* ms_out);

/* GEMM self-check (test infrastructure): tile variant `variant` (20-23: the
 * 256x256 phased kernel) against the 128x128 kernel on the same random operands,
 * fp32 C; mode 0 plain, 1 SwooshL, 2 residual.  Writes max |diff| and max |ref|. */
int zv_gemm_selftest(int M, int N, int K, int variant, int mode, float* maxdiff, float* maxref);

/* Attention plan (host only, no GPU; test infrastructure): the LDS bytes of the fused
 * attention consumers a layer of sequence length L would launch — SelfAttention (sa_plo < 0:
 * the plain kernel, 0 / 1: the Toeplitz kernel without / with the table's lo half),
 * NonlinAttention of value width nv_na with scoring form tpm, the head-0 statistics — and
 * whether the fused path is taken (fits = 1) or the W-materialising fallback (0).
 * tpm = 3: the second-generation set of the bf16 / fp8 engines (zv_flash2.inc: base-2 scores,
 * no statistics pass, lds_stats = 0; sa_plo ignored).
 * split: 1 (16-bit operands) or 3 (fp32-accurate hi/lo). */
int zv_attn_plan(int split, int sa_plo, int tpm, int L, int nv_na, int64_t* lds_sa, int64_t* lds_na,
                 int64_t* lds_stats, int* fits);

/* MX-fp8 operand format of the fp8 mode (csrc/zv_mx8.inc): e4m3 values, one E8M0 scale byte per
 * 32 consecutive K elements.  zv_mx8_quantize: the host quantiser the engine applies to the
 * fp8 weights (host pointers, no GPU: x (rows, K) fp32 -> q (rows, ldq), s (rows, ldq / 32),
 * ldq = K rounded up to 128).  zv_mx8_gemm_check: the fp8 GEMM end to end on the device (host
 * pointers in and out): A (M, K) is rounded to bf16 and quantised by the device producer kernel
 * (zv_mx8_pack_kernel; its output returned in Aq / As), W (N, K) by the host quantiser, and
 * C = A8 . W8^T through the block-scaled MFMA GEMM with the residual epilogue (zero residual
 * and bias), K a multiple of 128.  Both replace no reference interface: they pin the fp8
 * mode's operand format and GEMM against tests/ (numpy). */
int zv_mx8_quantize(const float* x, int rows, int K, uint8_t* q, uint8_t* s);
int zv_mx8_gemm_check(int M, int N, int K, const float* A, const float* W, float* C, uint8_t* Aq,
                      uint8_t* As);

/* Raw decoder: v = fm_decoder(cat[xt, text_c, speech_c], t, pad, g).
 *  t:      [N] timesteps;  guidance: [N] (distill only, else NULL)
 *  xt, speech_c: [N, T, Fx]; text_c: [N, T, feat_dim]; pad: [N, T] uint8 (1 = padded) or NULL
 *  v_out:  [N, T, Fout] with Fout = Fx (stereo: stream chosen by input width). */
int zv_fm_decoder(zv_handle h, const float* t, const float* guidance, const float* xt,
                  const float* text_c, const float* speech_c, const uint8_t* pad, int N,
                  int T, int Fx, float* v_out, void* stream);

/* One guided velocity evaluation (solver.py:40-165): CFG doubling inside,
 * x/text_c/speech_c/pad are the B un-doubled rows; v_out [B, T, Fx]. */
int zv_velocity(zv_handle h, float t, float guidance_scale, const float* x,
                const float* text_c, const float* speech_c, const uint8_t* pad, int B, int T,
                float* v_out, void* stream);

/* Full Euler ODE solve (solver.py:182-240), in place: x holds x0 on entry and
 * x(t_end) on return.  Time grid: t_shift*u/(1+(t_shift-1)u), u = linspace. */
int zv_euler_sample(zv_handle h, float* x, const float* text_c, const float* speech_c,
                    const uint8_t* pad, int B, int T, int num_step, float guidance_scale,
                    float t_start, float t_end, float t_shift, void* stream);

/* Per-utterance guidance scales (the reference's guidance_scale tensor of shape
 * (batch, 1, 1), solver.py:61-62): guidance_rows is a device array of B floats.
 * (guidance_rows == 0).all() selects the unguided branch (solver.py:71-79; one small
 * device-to-host read at entry, as the reference's host predicate); otherwise CFG with
 * g_b per row, doubled where t <= 0.5 (:95).  Distill: the rows feed the guidance
 * embedding (solver.py:127-165). */
int zv_velocity_rows(zv_handle h, float t, const float* guidance_rows, const float* x,
                     const float* text_c, const float* speech_c, const uint8_t* pad, int B,
                     int T, float* v_out, void* stream);
int zv_euler_sample_rows(zv_handle h, float* x, const float* text_c, const float* speech_c,
                         const uint8_t* pad, int B, int T, int num_step,
                         const float* guidance_rows, float t_start, float t_end,
                         float t_shift, void* stream);

/* Text encoder (+ dialog speaker-turn embeddings).
 *  tokens: [B, S] int64 (already padded with pad_id, one extra pad per row);
 *  pad: [B, S] uint8; spk: [B, S] int8 in {-1,0,1} (dialog only, else NULL);
 *  out: [B, S, feat_dim]. */
int zv_text_encode(zv_handle h, const int64_t* tokens, const uint8_t* pad,
                   const int8_t* spk, int B, int S, float* out, void* stream);

/* Frame-rate text condition: out[b, f] = embed[b, min(f / (T_b / S_b), S_b)].
 *  tok_lens, feat_lens: [B] int32 device; out: [B, T, feat_dim]. */
int zv_text_condition(zv_handle h, const float* embed, int B, int S, const int32_t* tok_lens,
                      const int32_t* feat_lens, int T, float* out, void* stream);

/* Speech condition: prompt features [B, Tp, F] padded/zeroed to [B, T, F]. */
int zv_speech_condition(zv_handle h, const float* prompt, int B, int Tp, int F,
                        const int32_t* prompt_lens, int T, float* out, void* stream);

/* ------------------------------------------------------------------------
 * Vocoder (Vocos, mel-24khz configuration: n_mels 100, dim 512, intermediate 1536,
 * 8 ConvNeXt blocks, ISTFT head n_fft 1024 / hop 256 / padding "same").
 * ---------------------------------------------------------------------- */
typedef struct zv_vocoder* zv_vocoder_handle;

/* Mirrors the vocos config.yaml backbone / head init_args. */
typedef struct {
  int precision;          /* zv_precision (ZV_FP32 = split-bf16x3 GEMMs, the parity mode) */
  int n_mels;             /* backbone.input_channels (100) */
  int dim;                /* backbone.dim (512) */
  int intermediate_dim;   /* backbone.intermediate_dim (1536) */
  int num_layers;         /* backbone.num_layers (8) */
  int n_fft;              /* head.n_fft (1024) */
  int hop;                /* head.hop_length (256) */
  int embed_kernel;       /* backbone.embed kernel size (7) */
  int dw_kernel;          /* ConvNeXt depthwise kernel size (7) */
} zv_vocoder_config;

zv_vocoder_handle zv_vocoder_create(const zv_vocoder_config* cfg);
void zv_vocoder_destroy(zv_vocoder_handle v);
/* Stage one vocos state-dict tensor (e.g. "backbone.convnext.3.pwconv1.weight",
 * "head.istft.window"); "feature_extractor.*" buffers are accepted and ignored. */
int zv_vocoder_set_weight(zv_vocoder_handle v, const char* name, const float* host_data,
                          int64_t numel);
int zv_vocoder_finalize(zv_vocoder_handle v);
/* wav[b, :T*hop] = decode(mel_b) for B utterances of up to T frames.
 *  layout 0: mel [B, n_mels, T] (Vocos.decode input, used as is: pass feat_scale 1, feat_bias 0);
 *  layout 1: model output [B, T, n_mels], post-processed as x / feat_scale - feat_bias
 *            (infer_zipvoice.py:374) inside the first kernel.
 *  lens: [B] int32 device frame counts (NULL = all T): utterance b is decoded on its own
 *        first lens[b] frames, exactly as a separate call would, and samples from
 *        lens[b]*hop on are 0.
 *  clamp: 1 applies clamp(-1, 1) (infer_zipvoice.py:378).  wav: [B, T*hop] fp32. */
int zv_vocoder_decode(zv_vocoder_handle v, const float* mel, int layout, float feat_scale,
                      float feat_bias, const int32_t* lens, int B, int T, float* wav, int clamp,
                      void* stream);
int64_t zv_vocoder_device_bytes(zv_vocoder_handle v);

/* ------------------------------------------------------------------------
 * Vocoder (BigVGAN-v2, bigvgan_v2_24khz_100band_256x), the one the reference loads for
 * feature.type "bigvgan_v2" (zipvoice/bin/infer_zipvoice.py:261-269: third-party
 * bigvgan.BigVGAN.from_pretrained(..., use_cuda_kernel=False) + remove_weight_norm();
 * decode(mel) = forward(mel)).  Weights are the weight-norm-removed state dict.
 * ---------------------------------------------------------------------- */
typedef struct zv_bigvgan* zv_bigvgan_handle;

/* Mirrors the bigvgan config.json fields the generator reads. */
typedef struct {
  int precision;                    /* zv_precision (ZV_FP32 = split-bf16x3 GEMMs) */
  int num_mels;                     /* 100 */
  int upsample_initial_channel;     /* 1536 */
  int num_upsamples;                /* len(upsample_rates) (6), <= 8 */
  int upsample_rates[8];            /* 4 4 2 2 2 2 */
  int upsample_kernel_sizes[8];     /* 8 8 4 4 4 4 */
  int num_kernels;                  /* len(resblock_kernel_sizes) (3), <= 3 */
  int resblock_kernel_sizes[3];     /* 3 7 11 */
  int resblock_dilation_sizes[3][3];/* (1 3 5) x 3; resblock "1" (AMPBlock1) */
  int snake_logscale;               /* 1 */
  int use_tanh_at_final;            /* 0: clamp(-1, 1) */
  int use_bias_at_final;            /* 0 */
} zv_bigvgan_config;

zv_bigvgan_handle zv_bigvgan_create(const zv_bigvgan_config* cfg);
void zv_bigvgan_destroy(zv_bigvgan_handle v);
/* Stage one generator tensor ("conv_pre.weight", "ups.0.0.weight",
 * "resblocks.4.convs1.2.bias", "resblocks.4.activations.3.act.alpha",
 * "activation_post.act.beta", "conv_post.weight", ...); the alias-free filter buffers
 * (*.upsample.filter, *.downsample.lowpass.filter) are accepted and checked. */
int zv_bigvgan_set_weight(zv_bigvgan_handle v, const char* name, const float* host_data,
                          int64_t numel);
int zv_bigvgan_finalize(zv_bigvgan_handle v);
/* wav[b, :T*hop] = forward(mel_b), hop = prod(upsample_rates); arguments as
 * zv_vocoder_decode (layout 0 [B, num_mels, T] / 1 [B, T, num_mels] with
 * x / feat_scale - feat_bias; lens [B] device frame counts or NULL).  The final
 * clamp (or tanh) is part of the network. */
int zv_bigvgan_decode(zv_bigvgan_handle v, const float* mel, int layout, float feat_scale,
                      float feat_bias, const int32_t* lens, int B, int T, float* wav,
                      void* stream);
int64_t zv_bigvgan_device_bytes(zv_bigvgan_handle v);

/* ------------------------------------------------------------------------
 * Prompt feature extractor (VocosFbank: centred reflect-padded STFT, power 1,
 * mel projection, log(clamp(1e-7)); fp32 arithmetic throughout).
 * ---------------------------------------------------------------------- */
typedef struct zv_fbank* zv_fbank_handle;
/* host_window: [n_fft] analysis window (torch.hann_window, periodic);
 * host_fb: [n_fft/2 + 1, n_mels] mel filterbank (torchaudio melscale_fbanks layout). */
zv_fbank_handle zv_fbank_create(int n_fft, int hop, int n_mels, const float* host_window,
                                const float* host_fb);
void zv_fbank_destroy(zv_fbank_handle f);
/* wav: [B, wav_ld] fp32 device samples, lens: [B] int32 sample counts (> n_fft/2);
 * out: [B, T_out, out_ld] log-mel rows (columns [0, n_mels)); utterance b fills its
 * first (lens[b] + hop/2) / hop rows (lhotse compute_num_frames), later rows are 0. */
/* Front-end variant (defaults: VocosFbank).  frame_offset = sample offset of frame
 * 0 (n_fft/2: centred STFT; (n_fft - hop)/2: BigVGANFbank's explicit reflect pad +
 * center=False), mag_eps added under the magnitude's square root (BigVGAN 1e-9),
 * log_floor the clamp before the log (Vocos 1e-7, BigVGAN 1e-5).  Frames past the
 * last STFT frame replicate it (BigVGANFbank's replicate pad to the lhotse count).
 * Reference: zipvoice/utils/feature.py:133-204, _bigvgan_mel_feature.py:42-111. */
int zv_fbank_configure(zv_fbank_handle f, int frame_offset, float mag_eps, float log_floor);
int zv_fbank_extract(zv_fbank_handle f, const float* wav, int64_t wav_ld, const int32_t* lens,
                     int B, int T_out, float* out, int64_t out_ld, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ZIPVOICE_HIP_H */
