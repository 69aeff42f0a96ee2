// Host launch entry points of the gfx950 kernels (defined in csrc/kernels/*.hip).
//
// Every kernel source is compiled once per 16-bit compute type (common.h): the bf16 build defines these in
// namespace pva_bf16, the fp16 build in namespace pva_f16.  This file has no include guard and no includes: the
// bindings include it inside each namespace (after conv_params.h and the HIP runtime header).
void conv_igemm_launch(const ConvParams& p, int chunk, hipStream_t stream, int cfg);
int conv_cfg_bm(int cfg, int N);
int conv_igemm_ut_legal(const ConvParams& p, int chunk, int bk);
int conv_direct_legal(const ConvParams& p, int chunk);
int conv_pw_legal(const ConvParams& p, int chunk);
int conv_halo_legal(const ConvParams& p, int chunk);
int conv_halo_epi_ok(const ConvParams& p);
int conv_halo64p_legal(const ConvParams& p, int chunk);
void conv_igemm_set_ut(int mode);
int conv_igemm_m_tiles(int M, int N);
int conv_igemm_m_tiles_k(int M, int N, int K, int Cg);
void conv_igemm_set_bk(int bk);
void conv_wgrad_launch(const WgradParams& p, int chunk, hipStream_t stream);
void conv_wgrad_tile(int Cout, int K, int variant, int* bmw, int* bnw);
int wgrad_rt_legal(int Cout, int Cin, int ldd, int ldx, int chunk, int dy_affine);
int wgrad_narrow_legal(int Cout, int Cin, int K);
int wgrad_halo_legal(const WgradParams& p);
int wgrad_box_legal(const WgradParams& p);
void wgrad_box_reduce_launch(const float* slab, float* tmp, float* grad, int splits, int Cout, int taps, int Cin,
                             int Cin_real, float scale, float beta, hipStream_t st);
int wgrad_box_reduce_groups(int splits);
void wgrad_reduce_launch(float* accbuf, float* grad, int splits, int Cout, int taps, int Cin, int Cin_real,
                         float scale, float beta, int slab, hipStream_t stream);
void bn_finalize_launch(const float* part, int tiles, int C, int64_t count, const float* gamma, const float* beta,
                        float* rm, float* rv, int64_t* nbt, float momentum, float eps, float* smean, float* srstd,
                        float* scale, float* shift, hipStream_t s, double* scratch, unsigned* ctr);
int bn_fin_ranges(int tiles);
void bn_eval_affine_launch(int C, const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                           float* scale, float* shift, hipStream_t s);
void bn_act_launch(const uint16_t* y, int ldy, uint16_t* out, int ldo, const float* scale, const float* shift,
                   int relu, int64_t M, int C, hipStream_t s);
void res_out_launch(const uint16_t* yc, const float* sc, const float* hc, const uint16_t* y1, const float* s1,
                    const float* h1, const uint16_t* x, int ldx, uint16_t* out, int ldo, uint8_t* mask, int64_t M,
                    int C, hipStream_t s);
int bn_bwd_reduce_blocks(int64_t M, int C, int* rows_per_block);
void bn_bwd_reduce_launch(const uint16_t* g, int ldg, int mask_mode, const void* mo, int ldm, const float* ms,
                          const float* mh, const uint16_t* y0, const float* mean0, const float* rstd0,
                          const uint16_t* y1, const float* mean1, const float* rstd1, int64_t M, int C, int blocks,
                          int rows_per_block, float* part, uint16_t* dzout, int lddz, hipStream_t s);
void bn_bwd_finalize_launch(const float* part, int blocks, int C, int64_t count, int which, const float* gamma,
                            const float* mean, const float* rstd, float* dgamma, float* dbeta, float beta_acc,
                            float* coef, hipStream_t s, double* scratch, unsigned* ctr);
void bn_bwd_apply_launch(const uint16_t* g, int ldg, int mask_mode, const void* mo, int ldm, const float* ms,
                         const float* mh, const uint16_t* y0, const float* coef0, uint16_t* dy0, const uint16_t* y1,
                         const float* coef1, uint16_t* dy1, uint16_t* dzout, int lddz, int dz_accum, int64_t M, int C,
                         hipStream_t s);
void stem_pool_fwd_launch(const uint16_t* y, const float* scale, const float* shift, uint16_t* out, uint8_t* arg,
                          uint16_t* ymax, int NT_, int H, int W, int Ho, int Wo, int C, int ldo, hipStream_t s);
void stem_pool_bn_apply_launch(const uint16_t* dout, int ldd, const uint8_t* arg, const uint16_t* y, const float* ms,
                               const float* mh, const float* coef, uint16_t* dy, int NT_, int H, int W, int Ho, int Wo,
                               int C, hipStream_t s);
int avgpool_global_splits(int N, int vol);
void stem_pool_bwd_launch(const uint16_t* dout, int ldd, const uint8_t* arg, uint16_t* dact, int NT_, int H, int W,
                          int Ho, int Wo, int C, hipStream_t s);
void avgpool_fwd_launch(const uint16_t* x, int N, int T, int H, int W, int C, int kt, int kh, int kw, float* out,
                        int ldo, int coff, float* scratch, hipStream_t s);
void avgpool_bwd_launch(const float* dout, int ldo, int coff, int N, int T, int H, int W, int C, int kt, int kh,
                        int kw, uint16_t* dx, hipStream_t s);
void sgd_momentum_launch(float* p, const float* g, float* buf, int64_t n, const float* lr, float momentum, float wd,
                         float gscale, int first, int* found_inf, const int* skip_flag, hipStream_t s);
void nonfinite_check_launch(const float* g, int64_t n, float gscale, int* flag, hipStream_t s);
void pack_weights_launch(const float* master, uint16_t* fwd, uint16_t* dgr, const void* descs, int ntensors,
                         hipStream_t s);
int pack_desc_size();
void video_preprocess_launch(const uint8_t* frames, const int* desc, const int* tidx, int B, int T, int S,
                             const float* mean, const float* std_, uint16_t* out, int s2d, hipStream_t s,
                             const int* slow_of = nullptr, uint16_t* slow_out = nullptr, int Ts = 0);
int stem_tiles(int Ho, int Wo, int N);
void stem_s2d_launch(int mode, const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, const uint16_t* dy,
                     float* dw, int N, int T, int Hs, int Ws, int Cout, int kt, hipStream_t s, float* slab = nullptr);
bool stem_s2d_supported(int Cout, int kt);
void stem_wgrad_convert_launch(float* acc, float* grad, int Cout, int kt, float beta, hipStream_t s);
void stem_pack_launch(const float* w, uint16_t* out, int Cout, int kt, hipStream_t s);
void synth_frames_launch(uint8_t* out, int64_t n, uint32_t seed, hipStream_t s);

void bnfold_fwd_stats_launch(const uint16_t* Wf, const float* Ga, const float* sslab, int splits, int C, int c,
                             int64_t count, float* T, float* s_out, const float* gamma, const float* beta, float* rm,
                             float* rv, int64_t* nbt, float momentum, float eps, float* smean, float* srstd,
                             float* scale, float* shift, hipStream_t st);
void bnfold_bwd_launch(const float* part, int tiles, const uint16_t* Wf, const uint16_t* Wd, const float* G,
                       const float* T, const float* s, int C, int c, int64_t count, const float* gamma,
                       const float* mean, const float* rstd, float* dgamma, float* dbeta, float* dW, float beta_acc,
                       float* coef, uint16_t* W1t, uint16_t* W2, float* bias, hipStream_t st);
void head_forward_launch(const float* feat, int N, int P, int C, const float* W, const float* b, int K, float p_drop,
                         uint64_t seed, const uint64_t* seedp, float* xm, float* logits, hipStream_t s);
void head_seed_advance_launch(uint64_t* seed, hipStream_t s);
void head_ce_launch(const float* logits, const int64_t* labels, int N, int K, float gscale, float* dlogits,
                    float* row_loss, int* row_correct, float* loss, int64_t* counts, int acc_counts, hipStream_t s);
void head_backward_launch(const float* dlogits, const float* xm, const float* W, int N, int P, int C, int K,
                          float p_drop, uint64_t seed, const uint64_t* seedp, float* dW, float* db, float beta,
                          float* dfeat, float* dlT, float* xmT, float* WT, hipStream_t s);
void head_dropout_mask_launch(int64_t total, float p_drop, uint64_t seed, uint8_t* out, hipStream_t s);
int lateral_bwd_legal(int CO, int Cf, int alpha, int To, int Tf, int kt, int pad);
void lateral_bwd_launch(const uint16_t* g, int ldg, const uint16_t* y, const float* sc, const float* sh,
                        const float* coef, const uint16_t* wd, uint16_t* dy, uint16_t* dx, int ldx, int N, int To,
                        int Tf, int HW, int CO, int Cf, int alpha, hipStream_t s);
int narrow_c_bwd_legal(int CO, int CI);
int narrow_c_bwd_rps(int64_t M, int CO, int splits);
void narrow_c_bwd_launch(const uint16_t* g, int ldg, int mode, const uint8_t* mask, const uint16_t* yc,
                         const float* coef, uint16_t* dz, int lddz, int dz_accum, const uint16_t* yb, const float* sb,
                         const float* hb, const float* mb, const float* rb, const uint16_t* wc, uint16_t* dab, int ldo,
                         int accum, float* slab, float* part, const uint16_t* y1, const float* mc, const float* rc,
                         const float* m1, const float* r1, float* cpart, int form, int64_t M, int CO, int CI, int rps,
                         hipStream_t s);
