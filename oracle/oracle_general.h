/*
 * oracle_general.h — TEST INFRASTRUCTURE ONLY.  Included by oracle_impl.h (once per REAL type).
 *
 * Restatement of the reference's GENERAL IFT path (core/tube_mpc.py:40-663): softplus / tanh
 * parameterised weights and DBaS parameters (core/params.py:9-59), the ancillary and nominal IFT
 * gradients of core/ift.py:35-92 in closed form, the reference-trajectory gradients that drive the
 * nominal sensitivity (core/tube_mpc.py:509-554), the clipped / momentum / projected update
 * (:239-255) and the plant step with the updated parameters (:589-600).  Also the receding-horizon
 * nominal MPC driver of run_nominal.py:204-415 (oracle_nominal_receding, at the end).
 *
 * Closed forms of the autograd quantities (per step k < N, with x' = f(x_k, u_k)):
 *   cost:      d/dQ_i [l_x . dx_k] = 2 (x_k - r_k)_i dx_k,i,  d/dR_j [l_u . du_k] = 2 (u_k - q_k)_j du_k,j,
 *              d/dqb = 2 b_k db_k (+ terminal), d/dQf_i = 2 (x_N - r_N)_i dx_N,i,
 *              d/dr_k = -2 Q (.) dx_k (terminal -2 Qf (.) dx_N), d/dq_k = -2 R (.) du_k
 *   dynamics:  dlam_{k+1,b} * d b'/d theta with b' = B(h(x') - s) - gamma (B(h(x_k) - s) - b_k):
 *              d b'/d gamma = -(B(h(x_k) - s) - b_k)
 *              d b'/d a     = dB/da(h(x') - s) - gamma dB/da(h(x_k) - s),  a = max(alpha, eps),
 *                             dB/da(z) = 0 on the safe branch z >= a, -3 (z - a)^2 / a^4 otherwise
 *              d b'/d s     = -B'(h(x') - s) + gamma B'(h(x_k) - s)
 *   chain:     softplus'(x) = e^x / (e^x + 1) (1 above torch's threshold 20), tanh' = 1 - tanh^2,
 *              d max(alpha, eps) / d alpha = 1 (alpha > eps), 1/2 (tie), 0 otherwise.
 *   xi term:   xi = x_hat0.detach() (core/tube_mpc.py:497) contributes nothing.
 */

#define GPAR_T CAT(ogpar, SUFFIX)

typedef struct {
  REAL Q[3], R[2], Qf[3], qb, alpha, gamma, tight;
  REAL dQ[3], dR[2], dQf[3], dqb, dalpha, dgamma, dtight; /* d value / d raw */
} GPAR_T;

/* torch.nn.functional.softplus(x) (beta 1, threshold 20) and its backward */
static REAL FN(softplus)(REAL x) { return x > (REAL)20 ? x : M_LOG1P(M_EXP(x)); }
static REAL FN(softplus_d)(REAL x) {
  if (x > (REAL)20) return (REAL)1;
  REAL z = M_EXP(x);
  return z / (z + (REAL)1);
}

/* core/params.py:28-35 (NominalTheta) / :49-56 (AuxiliaryTheta) */
static void FN(gpar_from)(const REAL* raw, int nominal, GPAR_T* p) {
  for (int i = 0; i < 3; ++i) {
    p->Q[i] = FN(softplus)(raw[DTMPC_P_Q + i]);
    p->dQ[i] = FN(softplus_d)(raw[DTMPC_P_Q + i]);
    p->Qf[i] = FN(softplus)(raw[DTMPC_P_QF + i]);
    p->dQf[i] = FN(softplus_d)(raw[DTMPC_P_QF + i]);
  }
  for (int j = 0; j < 2; ++j) {
    p->R[j] = FN(softplus)(raw[DTMPC_P_R + j]);
    p->dR[j] = FN(softplus_d)(raw[DTMPC_P_R + j]);
  }
  p->qb = FN(softplus)(raw[DTMPC_P_QB]);
  p->dqb = FN(softplus_d)(raw[DTMPC_P_QB]);
  p->alpha = FN(softplus)(raw[DTMPC_P_ALPHA]) + (REAL)1e-6;
  p->dalpha = FN(softplus_d)(raw[DTMPC_P_ALPHA]);
  p->gamma = M_TANH(raw[DTMPC_P_GAMMA]);
  p->dgamma = (REAL)1 - p->gamma * p->gamma;
  if (nominal) {
    p->tight = FN(softplus)(raw[DTMPC_P_TIGHT]);
    p->dtight = FN(softplus_d)(raw[DTMPC_P_TIGHT]);
  } else {
    p->tight = 0;
    p->dtight = 0;
  }
}

/* spec of a solve with the parameterised DBaS (core/tube_mpc.py:134-149, 230-238, 347-355) */
static void FN(gspec)(const SPEC_T* base, const GPAR_T* p, SPEC_T* o) {
  *o = *base;
  o->alpha = p->alpha;
  o->gamma = p->gamma;
  o->tight = p->tight;
}

/* cost with the parameterised weights: nominal (:240-256) or ancillary (:358-379, terminal Qf) */
static void FN(gcost)(const GPAR_T* p, int kind, const double* target, COST_T* c) {
  c->kind = kind;
  c->wrap = 0;
  for (int i = 0; i < 3; ++i) {
    c->Q[i] = p->Q[i];
    c->Qf[i] = p->Qf[i];
    c->target[i] = kind == DTMPC_COST_TARGET ? (REAL)target[i] : (REAL)0;
  }
  c->R[0] = p->R[0];
  c->R[1] = p->R[1];
  c->qb = p->qb;
}

/* dB/dz of the dynamics barrier (autograd of core/barrier.py:36-72) */
static REAL FN(dbarrier_dyn)(const SPEC_T* s, REAL z) {
  if (s->barrier == DTMPC_BARRIER_LOG) return z >= s->eps ? (REAL)(-1) / z : (REAL)0;
  return FN(dbarrier_relaxed)(s, z);
}

/* dB_alpha/d alpha_eff of the relaxed inverse barrier (core/barrier.py:52-59) */
static REAL FN(dbarrier_da)(const SPEC_T* s, REAL z) {
  if (s->barrier == DTMPC_BARRIER_LOG) return (REAL)0;
  REAL a = s->alpha > s->eps ? s->alpha : s->eps;
  if (z >= a) return (REAL)0;
  REAL d = z - a;
  REAL a2 = a * a;
  return (REAL)(-3) * (d * d) / (a2 * a2);
}

/* ift_gradient core/ift.py:35-92 with the closures of core/tube_mpc.py:461-500 (TRACK) or
 * :556-585 (TARGET).  s: spec with the parameterised alpha / gamma / tight (FN(gspec)).
 * g[12] (raw layout DTMPC_P_*), gxr [(N+1)*3] and gur [N*2] (TRACK; may be NULL). */
static void FN(ift1)(const SPEC_T* s, const COST_T* c, const GPAR_T* p, const REAL* X, const REAL* V,
                     const REAL* dX, const REAL* dV, const REAL* dl, const REAL* Xr, const REAL* Ur,
                     REAL* g, REAL* gxr, REAL* gur) {
  int N = s->N;
  int track = c->kind == DTMPC_COST_TRACK;
  REAL gQ[3] = {0, 0, 0}, gR[2] = {0, 0}, gQf[3] = {0, 0, 0}, gqb = 0, ga = 0, gg = 0, gs = 0;
  for (int k = 0; k < N; ++k) {
    const REAL* xk = X + 4 * k;
    const REAL* uk = V + 2 * k;
    const REAL* dxk = dX + 4 * k;
    const REAL* duk = dV + 2 * k;
    for (int i = 0; i < 3; ++i) {
      REAL d = xk[i] - (track ? Xr[3 * k + i] : c->target[i]);
      gQ[i] += (REAL)2 * d * dxk[i];
      if (track && gxr) gxr[3 * k + i] = -((REAL)2 * p->Q[i]) * dxk[i];
    }
    for (int j = 0; j < 2; ++j) {
      REAL e = uk[j] - (track ? Ur[2 * k + j] : (REAL)0);
      gR[j] += (REAL)2 * e * duk[j];
      if (track && gur) gur[2 * k + j] = -((REAL)2 * p->R[j]) * duk[j];
    }
    gqb += (REAL)2 * xk[3] * dxk[3];
    /* dynamics term: dlam_{k+1} . f_hat(x_k, u_k; theta), only b' depends on theta */
    REAL lam = dl[4 * (k + 1) + 3];
    REAL xn[3], gx, gy;
    FN(dubins)(s, xk, uk, xn);
    REAL hn = FN(h_eval)(s, xn[0], xn[1], &gx, &gy) - s->tight;
    REAL hc = FN(h_eval)(s, xk[0], xk[1], &gx, &gy) - s->tight;
    REAL Bc = FN(barrier_dyn)(s, hc);
    gg += lam * (-(Bc - xk[3]));
    ga += lam * (FN(dbarrier_da)(s, hn) - s->gamma * FN(dbarrier_da)(s, hc));
    gs += lam * (-FN(dbarrier_dyn)(s, hn) + s->gamma * FN(dbarrier_dyn)(s, hc));
  }
  const REAL* xN = X + 4 * N;
  const REAL* dxN = dX + 4 * N;
  for (int i = 0; i < 3; ++i) {
    REAL d = xN[i] - (track ? Xr[3 * N + i] : c->target[i]);
    gQf[i] += (REAL)2 * d * dxN[i];
    if (track && gxr) gxr[3 * N + i] = -((REAL)2 * p->Qf[i]) * dxN[i];
  }
  gqb += (REAL)2 * xN[3] * dxN[3];
  REAL dmax = p->alpha > s->eps ? (REAL)1 : (p->alpha == s->eps ? (REAL)0.5 : (REAL)0);
  for (int i = 0; i < 3; ++i) {
    g[DTMPC_P_Q + i] = gQ[i] * p->dQ[i];
    g[DTMPC_P_QF + i] = gQf[i] * p->dQf[i];
  }
  g[DTMPC_P_R] = gR[0] * p->dR[0];
  g[DTMPC_P_R + 1] = gR[1] * p->dR[1];
  g[DTMPC_P_QB] = gqb * p->dqb;
  g[DTMPC_P_ALPHA] = ga * dmax * p->dalpha;
  g[DTMPC_P_GAMMA] = gg * p->dgamma;
  g[DTMPC_P_TIGHT] = track ? (REAL)0 : gs * p->dtight;
}

/* One trajectory of the general loop body up to the gradients (core/tube_mpc.py:217-584).
 * xs/bs: plant state, xb/bb: nominal state.  Vn/Va: warm starts in, optima out.
 * gout[24] = L, g_theta(11), g_theta_bar(12).  work: see oracle_general_step. */
static int FN(general1)(const SPEC_T* s0, const dtmpc_general_cfg* cfg, const GPAR_T* pa, const GPAR_T* pn,
                        const REAL* xs, REAL bs, const REAL* xb, REAL bb, REAL* Xn, REAL* Vn, REAL* Xa,
                        REAL* Va, REAL* gout, int* itn, int* ita, REAL* work) {
  int N = s0->N;
  SPEC_T sn, sa;
  COST_T cn, ca;
  FN(gspec)(s0, pn, &sn);
  FN(gspec)(s0, pa, &sa);
  FN(gcost)(pn, DTMPC_COST_TARGET, cfg->target, &cn);
  FN(gcost)(pa, DTMPC_COST_TRACK, cfg->target, &ca);
  REAL* Xr = work;                  /* (N+1)*3 */
  REAL* K = Xr + 3 * (N + 1);       /* 8N */
  REAL* kf = K + 8 * N;             /* 2N */
  REAL* wk = kf + 2 * N;            /* 2*(4(N+1) + 2N) */
  REAL* dXa = wk + 2 * (4 * (N + 1) + 2 * N);
  REAL* dVa = dXa + 4 * (N + 1);
  REAL* dla = dVa + 2 * N;
  REAL* gxr = dla + 4 * (N + 1);    /* (N+1)*3 */
  REAL* gur = gxr + 3 * (N + 1);    /* 2N */
  REAL* gX = gur + 2 * N;           /* (N+1)*4 */
  REAL* dXn = gX + 4 * (N + 1);
  REAL* dVn = dXn + 4 * (N + 1);
  REAL* dln = dVn + 2 * N;
  REAL* wk2 = dln + 4 * (N + 1);    /* sens1 scratch */
  int st = 0;
  REAL x0[4] = {xb[0], xb[1], xb[2], bb};
  st |= FN(ilqr1)(&sn, &cn, &cfg->nom_ilqr, x0, NULL, NULL, Xn, Vn, K, kf, itn, wk, NULL, 0, NULL);
  for (int k = 0; k <= N; ++k)
    for (int f = 0; f < 3; ++f) Xr[3 * k + f] = Xn[4 * k + f];
  x0[0] = xs[0];
  x0[1] = xs[1];
  x0[2] = xs[2];
  x0[3] = bs;
  st |= FN(ilqr1)(&sa, &ca, &cfg->aux_ilqr, x0, Xr, Vn, Xa, Va, K, kf, ita, wk, NULL, 0, NULL);
  /* upper loss L = ||x* - xbar||^2 + ||b*||^2 (:403-408) */
  REAL L1 = 0, L2 = 0;
  for (int k = 0; k <= N; ++k) {
    for (int i = 0; i < 3; ++i) {
      REAL d = Xa[4 * k + i] - Xn[4 * k + i];
      L1 += d * d;
    }
    L2 += Xa[4 * k + 3] * Xa[4 * k + 3];
  }
  for (int j = 0; j < DTMPC_GEN_SUMS; ++j) gout[j] = 0;
  gout[0] = L1 + L2;
  /* ancillary sensitivity with the paper upper loss (:424-455) + IFT (:457-500) */
  st |= FN(sens1)(&sa, &ca, Xa, Va, Xr, Vn, Xr, NULL, NULL, dXa, dVa, dla, wk2);
  REAL ga[DTMPC_P_COUNT];
  FN(ift1)(&sa, &ca, pa, Xa, Va, dXa, dVa, dla, Xr, Vn, ga, gxr, gur);
  for (int j = 0; j < 11; ++j) gout[1 + j] = ga[j];
  if (cfg->adapt_nominal) {
    /* nominal sensitivity driven by [dL/dX_ref, 0], dL/dU_ref (:511-554) + IFT (:556-585) */
    for (int k = 0; k <= N; ++k) {
      for (int f = 0; f < 3; ++f) gX[4 * k + f] = gxr[3 * k + f];
      gX[4 * k + 3] = 0;
    }
    st |= FN(sens1)(&sn, &cn, Xn, Vn, NULL, NULL, NULL, gX, gur, dXn, dVn, dln, wk2);
    REAL gn[DTMPC_P_COUNT];
    FN(ift1)(&sn, &cn, pn, Xn, Vn, dXn, dVn, dln, NULL, NULL, gn, NULL, NULL);
    for (int j = 0; j < 12; ++j) gout[12 + j] = gn[j];
  }
  for (int j = 0; j < DTMPC_GEN_SUMS; ++j) st |= FN(isfin)(gout[j]) ? 0 : DTMPC_ST_NONFINITE;
  return st;
}

/* ---- exported ----------------------------------------------------------------------------- */

/* ddp_sensitivity with array upper gradients: gX [N+1][4][B], gU [N][2][B] (SoA) */
void FN(oracle_ddp_sensitivity_upper)(const dtmpc_spec* sp, const dtmpc_cost* cp, long long B,
                                      const REAL* X, const REAL* U, const REAL* gX, const REAL* gU,
                                      REAL* dX, REAL* dU, REAL* dlam, int* status) {
  SPEC_T s;
  COST_T c;
  FN(spec_from)(sp, &s);
  FN(cost_from)(cp, &c);
  int N = s.N;
  size_t per = (size_t)(4 * (N + 1) * 5 + 2 * N * 3 + 16 * N + 8 * N + 8 * N + 2 * N + 16 * (N + 1) +
                        4 * (N + 1) + 2 * N + 64);
  REAL* buf = (REAL*)malloc(sizeof(REAL) * per + sizeof(int) * 2 * N + 64);
  REAL* Xa = buf;
  REAL* Va = Xa + 4 * (N + 1);
  REAL* gx = Va + 2 * N;
  REAL* gu = gx + 4 * (N + 1);
  REAL* dXa = gu + 2 * N;
  REAL* dVa = dXa + 4 * (N + 1);
  REAL* dla = dVa + 2 * N;
  REAL* wk = dla + 4 * (N + 1);
  for (long long i = 0; i < B; ++i) {
    FN(gather)(X, N + 1, 4, B, i, Xa);
    FN(gather)(U, N, 2, B, i, Va);
    FN(gather)(gX, N + 1, 4, B, i, gx);
    FN(gather)(gU, N, 2, B, i, gu);
    int st = FN(sens1)(&s, &c, Xa, Va, NULL, NULL, NULL, gx, gu, dXa, dVa, dlam ? dla : NULL, wk);
    FN(scatter)(dXa, N + 1, 4, B, i, dX);
    FN(scatter)(dVa, N, 2, B, i, dU);
    if (dlam) FN(scatter)(dla, N + 1, 4, B, i, dlam);
    if (status) status[i] |= st;
  }
  free(buf);
}

/* ift_gradient for B trajectories (SoA in/out as dtmpc_ift_gradient) */
void FN(oracle_ift_gradient)(const dtmpc_spec* sp, const dtmpc_cost* cp, const double* theta_raw,
                             long long B, const REAL* X, const REAL* U, const REAL* dX, const REAL* dU,
                             const REAL* dlam, const REAL* Xref, const REAL* Uref, REAL* g_theta,
                             REAL* g_xref, REAL* g_uref) {
  SPEC_T s0, s;
  FN(spec_from)(sp, &s0);
  int N = s0.N;
  int track = cp->kind == DTMPC_COST_TRACK;
  REAL raw[DTMPC_P_COUNT];
  for (int j = 0; j < DTMPC_P_COUNT; ++j) raw[j] = (REAL)theta_raw[j];
  GPAR_T p;
  FN(gpar_from)(raw, !track, &p);
  FN(gspec)(&s0, &p, &s);
  COST_T c;
  FN(gcost)(&p, cp->kind, cp->target, &c);
  size_t per = (size_t)(4 * (N + 1) * 3 + 2 * N * 2 + 3 * (N + 1) * 2 + 2 * N * 2 + 16);
  REAL* buf = (REAL*)malloc(sizeof(REAL) * per);
  REAL* Xa = buf;
  REAL* Va = Xa + 4 * (N + 1);
  REAL* dXa = Va + 2 * N;
  REAL* dVa = dXa + 4 * (N + 1);
  REAL* dla = dVa + 2 * N;
  REAL* Xr = dla + 4 * (N + 1);
  REAL* Ur = Xr + 3 * (N + 1);
  REAL* gxr = Ur + 2 * N;
  REAL* gur = gxr + 3 * (N + 1);
  REAL g[DTMPC_P_COUNT];
  for (long long i = 0; i < B; ++i) {
    FN(gather)(X, N + 1, 4, B, i, Xa);
    FN(gather)(U, N, 2, B, i, Va);
    FN(gather)(dX, N + 1, 4, B, i, dXa);
    FN(gather)(dU, N, 2, B, i, dVa);
    FN(gather)(dlam, N + 1, 4, B, i, dla);
    if (track) {
      FN(gather)(Xref, N + 1, 3, B, i, Xr);
      FN(gather)(Uref, N, 2, B, i, Ur);
    }
    FN(ift1)(&s, &c, &p, Xa, Va, dXa, dVa, dla, Xr, Ur, g, gxr, gur);
    for (int j = 0; j < DTMPC_P_COUNT; ++j) g_theta[(long long)j * B + i] = g[j];
    if (track && g_xref) FN(scatter)(gxr, N + 1, 3, B, i, g_xref);
    if (track && g_uref) FN(scatter)(gur, N, 2, B, i, g_uref);
  }
  free(buf);
}

/* softplus-transformed parameters (for the logs: Qa_history = theta.Q(), core/tube_mpc.py:611-614) */
void FN(oracle_softplus)(long long n, const REAL* x, REAL* y) {
  for (long long i = 0; i < n; ++i) y[i] = FN(softplus)(x[i]);
}

/* general loop body up to the gradients for every trajectory (dtmpc_general_step).
 * theta [2][12] raw (row 0 ancillary, row 1 nominal).  gout [24][B]. */
void FN(oracle_general_step)(const dtmpc_spec* sp, const dtmpc_general_cfg* cfg, long long B, const REAL* x,
                             const REAL* b, const REAL* xbar, const REAL* bbar, REAL* Xnom, REAL* Unom,
                             REAL* Xaux, REAL* Uaux, const REAL* theta, REAL* gout, int* status, int* iters,
                             int nthreads) {
  SPEC_T s0;
  FN(spec_from)(sp, &s0);
  int N = s0.N;
  GPAR_T pa, pn;
  FN(gpar_from)(theta, 0, &pa);
  FN(gpar_from)(theta + DTMPC_P_COUNT, 1, &pn);
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    size_t per = (size_t)(2 * 4 * (N + 1) + 2 * 2 * N + 40 * (N + 1) + 40 * N + 16 * N + 8 * N + 8 * N +
                          2 * N + 16 * (N + 1) + 4 * (N + 1) + 2 * N + 256);
    REAL* buf = (REAL*)malloc(sizeof(REAL) * per + sizeof(int) * 2 * N + 64);
    REAL* Xn = buf;
    REAL* Vn = Xn + 4 * (N + 1);
    REAL* Xa = Vn + 2 * N;
    REAL* Va = Xa + 4 * (N + 1);
    REAL* wk = Va + 2 * N;
#pragma omp for schedule(dynamic, 1)
    for (long long i = 0; i < B; ++i) {
      REAL xs[3], xb[3], go[DTMPC_GEN_SUMS];
      for (int f = 0; f < 3; ++f) {
        xs[f] = x[(long long)f * B + i];
        xb[f] = xbar[(long long)f * B + i];
      }
      FN(gather)(Unom, N, 2, B, i, Vn);
      FN(gather)(Uaux, N, 2, B, i, Va);
      int itn = 0, ita = 0;
      int st = FN(general1)(&s0, cfg, &pa, &pn, xs, b[i], xb, bbar[i], Xn, Vn, Xa, Va, go, &itn, &ita, wk);
      FN(scatter)(Xn, N + 1, 4, B, i, Xnom);
      FN(scatter)(Vn, N, 2, B, i, Unom);
      FN(scatter)(Xa, N + 1, 4, B, i, Xaux);
      FN(scatter)(Va, N, 2, B, i, Uaux);
      /* L always (logged); gradients zero and healthy count 0 for a flagged trajectory */
      go[DTMPC_GEN_SUMS - 1] = 1;
      gout[i] = go[0];
      for (int j = 1; j < DTMPC_GEN_SUMS; ++j) gout[(long long)j * B + i] = st ? (REAL)0 : go[j];
      if (status) status[i] |= st;
      if (iters) {
        iters[i] = itn;
        iters[B + i] = ita;
      }
    }
    free(buf);
  }
}

/* _apply_update core/tube_mpc.py:239-255 on one parameter tensor (n elements) */
static void FN(apply_update)(const dtmpc_general_cfg* cfg, REAL inv_batch, const REAL* sums, REAL* p, REAL* v,
                             int n, int proj) {
  REAL g[3];
  for (int j = 0; j < n; ++j) g[j] = sums[j] * inv_batch;
  if (cfg->clip_norm > 0) {
    double nn = 0;
    REAL acc = 0;
    for (int j = 0; j < n; ++j) acc += g[j] * g[j];
    nn = (double)sqrt((double)acc);
    if (nn > cfg->clip_norm) {
      REAL sc = (REAL)(cfg->clip_norm / (nn + 1e-12));
      for (int j = 0; j < n; ++j) g[j] = g[j] * sc;
    }
  }
  for (int j = 0; j < n; ++j) {
    REAL stp;
    if (cfg->momentum > 0) {
      v[j] = v[j] * (REAL)cfg->momentum + g[j];
      stp = v[j];
    } else {
      stp = g[j];
    }
    REAL t = p[j] - (REAL)cfg->lr_eta * stp;
    if (cfg->project_params) {
      /* _project :192-237 */
      switch (proj) {
        case 0: t = t < 0 ? (REAL)0 : t; break;                                  /* Q, Qf */
        case 1: t = FN(clampv)(t, (REAL)1e-4, (REAL)1e4); break;                 /* R */
        case 2: t = FN(clampv)(t, (REAL)0, (REAL)1); break;                      /* qb, alpha */
        case 3: t = FN(clampv)(t, (REAL)(-1), (REAL)1); break;                   /* gamma */
        default: t = FN(clampv)(t, (REAL)0, (REAL)2); break;                     /* tight */
      }
    }
    p[j] = t;
  }
}

/* theta [2][12], vel [2][12], sums [24] (batch sums); barrier: the alpha gradient is None for the
 * log barrier (alpha unused in the graph), so alpha is not updated there (:243-244). */
void FN(oracle_general_update)(const dtmpc_spec* sp, const dtmpc_general_cfg* cfg, double inv_batch,
                               const REAL* sums, REAL* theta, REAL* vel) {
  REAL ib = (REAL)inv_batch;
  if (!(inv_batch > 0)) ib = sums[DTMPC_GEN_SUMS - 1] > 0 ? (REAL)1 / sums[DTMPC_GEN_SUMS - 1] : (REAL)0;
  int alpha_used = sp->barrier_type != DTMPC_BARRIER_LOG;
  if (cfg->adapt_ancillary) {
    const REAL* g = sums + 1;
    REAL* p = theta;
    REAL* v = vel;
    FN(apply_update)(cfg, ib, g + DTMPC_P_Q, p + DTMPC_P_Q, v + DTMPC_P_Q, 3, 0);
    FN(apply_update)(cfg, ib, g + DTMPC_P_R, p + DTMPC_P_R, v + DTMPC_P_R, 2, 1);
    FN(apply_update)(cfg, ib, g + DTMPC_P_QF, p + DTMPC_P_QF, v + DTMPC_P_QF, 3, 0);
    FN(apply_update)(cfg, ib, g + DTMPC_P_QB, p + DTMPC_P_QB, v + DTMPC_P_QB, 1, 2);
    if (alpha_used) FN(apply_update)(cfg, ib, g + DTMPC_P_ALPHA, p + DTMPC_P_ALPHA, v + DTMPC_P_ALPHA, 1, 2);
    FN(apply_update)(cfg, ib, g + DTMPC_P_GAMMA, p + DTMPC_P_GAMMA, v + DTMPC_P_GAMMA, 1, 3);
  }
  if (cfg->adapt_nominal) {
    const REAL* g = sums + 12;
    REAL* p = theta + DTMPC_P_COUNT;
    REAL* v = vel + DTMPC_P_COUNT;
    FN(apply_update)(cfg, ib, g + DTMPC_P_Q, p + DTMPC_P_Q, v + DTMPC_P_Q, 3, 0);
    FN(apply_update)(cfg, ib, g + DTMPC_P_R, p + DTMPC_P_R, v + DTMPC_P_R, 2, 1);
    FN(apply_update)(cfg, ib, g + DTMPC_P_QF, p + DTMPC_P_QF, v + DTMPC_P_QF, 3, 0);
    FN(apply_update)(cfg, ib, g + DTMPC_P_QB, p + DTMPC_P_QB, v + DTMPC_P_QB, 1, 2);
    if (alpha_used) FN(apply_update)(cfg, ib, g + DTMPC_P_ALPHA, p + DTMPC_P_ALPHA, v + DTMPC_P_ALPHA, 1, 2);
    FN(apply_update)(cfg, ib, g + DTMPC_P_GAMMA, p + DTMPC_P_GAMMA, v + DTMPC_P_GAMMA, 1, 3);
    FN(apply_update)(cfg, ib, g + DTMPC_P_TIGHT, p + DTMPC_P_TIGHT, v + DTMPC_P_TIGHT, 1, 4);
  }
}

/* plant + nominal propagation with the UPDATED theta (:589-600), log (:602-614), warm-start shift
 * (:616-621).  Unom/Uaux hold the optima of this step.  log [12][B] (may be NULL), L [B] (the
 * upper loss of the step, logged).  w [3][B] or NULL (Philox). */
void FN(oracle_general_plant)(const dtmpc_spec* sp, const dtmpc_general_cfg* cfg, long long B, long long goff,
                              long long step, REAL* x, REAL* b, REAL* xbar, REAL* bbar, REAL* Unom, REAL* Uaux,
                              const REAL* theta, const REAL* L, const REAL* w, REAL* log) {
  SPEC_T s0, sa, sn;
  FN(spec_from)(sp, &s0);
  int N = s0.N;
  GPAR_T pa, pn;
  FN(gpar_from)(theta, 0, &pa);
  FN(gpar_from)(theta + DTMPC_P_COUNT, 1, &pn);
  FN(gspec)(&s0, &pa, &sa);
  FN(gspec)(&s0, &pn, &sn);
  dtmpc_tube_cfg tc;
  memset(&tc, 0, sizeof(tc));
  tc.seed = cfg->seed;
  for (int f = 0; f < 3; ++f) {
    tc.w_low[f] = cfg->w_low[f];
    tc.w_high[f] = cfg->w_high[f];
  }
  for (long long i = 0; i < B; ++i) {
    REAL xh[4], xbh[4], u[2], ub[2], xn[4], xbn[4], ww[3];
    for (int f = 0; f < 3; ++f) {
      xh[f] = x[(long long)f * B + i];
      xbh[f] = xbar[(long long)f * B + i];
    }
    xh[3] = b[i];
    xbh[3] = bbar[i];
    for (int a = 0; a < 2; ++a) {
      u[a] = Uaux[(long long)a * B + i];
      ub[a] = Unom[(long long)a * B + i];
    }
    if (w) {
      for (int f = 0; f < 3; ++f) ww[f] = w[(long long)f * B + i];
    } else {
      FN(philox_w)(&tc, goff + i, step, ww);
    }
    FN(fhat)(&sa, xh, u, xn);
    FN(fhat)(&sn, xbh, ub, xbn);
    if (log) {
      for (int f = 0; f < 3; ++f) log[(long long)f * B + i] = xh[f];
      log[3 * B + i] = u[0];
      log[4 * B + i] = u[1];
      for (int f = 0; f < 3; ++f) log[(long long)(5 + f) * B + i] = xbh[f];
      log[8 * B + i] = ub[0];
      log[9 * B + i] = ub[1];
      log[10 * B + i] = xh[3];
      log[11 * B + i] = L[i];
    }
    for (int f = 0; f < 3; ++f) {
      x[(long long)f * B + i] = xn[f] + ww[f];
      xbar[(long long)f * B + i] = xbn[f];
    }
    b[i] = xn[3];
    bbar[i] = xbn[3];
    for (int k = 0; k + 1 < N; ++k)
      for (int a = 0; a < 2; ++a) {
        Unom[((long long)k * 2 + a) * B + i] = Unom[((long long)(k + 1) * 2 + a) * B + i];
        Uaux[((long long)k * 2 + a) * B + i] = Uaux[((long long)(k + 1) * 2 + a) * B + i];
      }
  }
}

#undef GPAR_T

/* ---- receding-horizon nominal MPC (run_nominal.py:204-415) ----------------------------------- */

/* true min_i h_i(x) over the circles (run_nominal.py:390-396; h_circle_obstacle :16-30) */
static REAL FN(h_true_min)(const SPEC_T* s, REAL px, REAL py) {
  REAL m = FN(h_circle)(s, 0, px, py);
  for (int i = 1; i < s->M; ++i) {
    REAL hi = FN(h_circle)(s, i, px, py);
    m = hi < m ? hi : m;
  }
  return m;
}

/* B independent receding-horizon runs from x0 [3][B] with warm starts Uws [N][2][B] (in: the
 * v = v_max rows of run_nominal.py:368-369; out: the last shifted plan).  log [H][6][B]: x(3), u0(2), b
 * per recorded step.  h_ran / success_t (-1 = none) / collided / status per trajectory. */
void FN(oracle_nominal_receding)(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cfg, long long B,
                                 int H, double success_r, const REAL* x0, REAL* Uws, REAL* log, int* h_ran,
                                 int* success_t, int* collided, int* status, int nthreads) {
  SPEC_T s;
  COST_T c;
  FN(spec_from)(sp, &s);
  FN(cost_from)(cp, &c);
  int N = s.N;
  int has_obs = s.agg != DTMPC_OBS_NONE && s.M > 0;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    size_t per = (size_t)(4 * (N + 1) + 2 * N + 8 * N + 2 * N + 2 * (4 * (N + 1) + 2 * N) + 16);
    REAL* buf = (REAL*)malloc(sizeof(REAL) * per);
    REAL* X = buf;
    REAL* V = X + 4 * (N + 1);
    REAL* K = V + 2 * N;
    REAL* kf = K + 8 * N;
    REAL* wk = kf + 2 * N;
#pragma omp for schedule(dynamic, 1)
    for (long long i = 0; i < B; ++i) {
      REAL xh[4], gx, gy;
      for (int f = 0; f < 3; ++f) xh[f] = x0[(long long)f * B + i];
      /* b = dbas_init_b0(x, h, db_cfg) (:279) */
      xh[3] = FN(barrier_dyn)(&s, FN(h_eval)(&s, xh[0], xh[1], &gx, &gy) - s.tight);
      FN(gather)(Uws, N, 2, B, i, V);
      int st = 0, ran = H, sidx = -1, coll = 0;
      for (int t = 0; t < H; ++t) {
        int it = 0;
        REAL x0h[4] = {xh[0], xh[1], xh[2], xh[3]};
        st |= FN(ilqr1)(&s, &c, cfg, x0h, NULL, NULL, X, V, K, kf, &it, wk, NULL, 0, NULL);
        REAL u0[2] = {V[0], V[1]}, xn[4];
        FN(fhat)(&s, xh, u0, xn);
        REAL rec[6] = {xh[0], xh[1], xh[2], u0[0], u0[1], xh[3]};
        for (int f = 0; f < 6; ++f) log[((long long)t * 6 + f) * B + i] = rec[f];
        if (st) {
          ran = t + 1;
          break;
        }
        if (has_obs && FN(h_true_min)(&s, xh[0], xh[1]) <= 0) { /* :388-397 */
          coll = 1;
          ran = t + 1;
          break;
        }
        REAL ex = xh[0] - c.target[0], ey = xh[1] - c.target[1];
        if (sqrt((double)(ex * ex + ey * ey)) <= success_r) { /* :399-403 */
          sidx = t;
          ran = t + 1;
          break;
        }
        for (int k = 0; k + 1 < N; ++k) { /* :405-406 */
          V[2 * k] = V[2 * (k + 1)];
          V[2 * k + 1] = V[2 * (k + 1) + 1];
        }
        for (int f = 0; f < 4; ++f) xh[f] = xn[f];
      }
      FN(scatter)(V, N, 2, B, i, Uws);
      h_ran[i] = ran;
      success_t[i] = sidx;
      collided[i] = coll;
      if (status) status[i] |= st;
    }
    free(buf);
  }
}
