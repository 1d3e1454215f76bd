/* CPU restatement of the reference weather-sim time step -- TEST INFRASTRUCTURE ONLY.
 *
 * Included twice by ws_oracle.c, once per scalar type (WS_T = float / double, WS_SFX =
 * f32 / f64). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load the resulting liboracle; the product (libws_hip.so) never does.
 *
 * It restates, statement by statement and with the same evaluation order and the same
 * loop / parallel structure, the reference CPU path (paths relative to
 * /root/reference/src/weather-sim/cpp):
 *   src/weather_simulation.cpp:117-158   step(): integrator dispatch, t += dt, step++,
 *                                        diagnostics on the new current grid
 *   src/weather_simulation.cpp:68-115    run() with the max_time break; runUntil()
 *   src/weather_simulation.cpp:160-218   stepExplicitEuler (+ PE T/P stale-tendency update)
 *   src/weather_simulation.cpp:220-323   stepRungeKutta2 (midpoint)
 *   src/weather_simulation.cpp:325-455   stepRungeKutta4 incl. the k1-aliases-tendency
 *                                        quirk (final uses k4 in place of k1) and the
 *                                        fallback to RK2 for non-SWE models (:334-338)
 *   src/weather_simulation.cpp:457-471   AdamsBashforth / SemiImplicit == Euler
 *   src/weather_simulation.cpp:473-540   computeShallowWaterTendencies (OpenMP collapse(2))
 *   src/weather_simulation.cpp:542-560   Barotropic / PE tendencies == SWE
 *   src/weather_grid.cpp:57-71           reset() defaults
 *   src/weather_grid.cpp:82-121          calculateDiagnostics (serial vorticity, divergence)
 * Grid rotation is the shared_ptr swap of current/next (weather_simulation.cpp:217,322,454),
 * so fields the stepper does not write alternate between the two grids.
 * The tendency grid is reset once at construction and only u,v,h are ever written, so its
 * T and P stay 288.15 / 1013.25 (weather_grid.cpp:63-65): the PE "stale tendency".
 * Build: -O3 -fopenmp -ffp-contract=off (no FMA contraction: bitwise parity).
 */

#define WS_CAT2(a, b) a##_##b
#define WS_CAT(a, b) WS_CAT2(a, b)
#define WS_FN(name) WS_CAT(ws_oracle, WS_CAT(WS_SFX, name))
#define WS_STATE WS_CAT(ws_oracle_state, WS_SFX)

typedef struct {
    WS_T *u, *v, *h, *p, *t, *q, *vort, *div;
} WS_CAT(ws_grid, WS_SFX);
#define WS_GRID WS_CAT(ws_grid, WS_SFX)

typedef struct {
    int W, H, model, method;
    WS_T dx, dy, dt, g, f, max_time;
    WS_T time;
    int step;
    WS_GRID g_[4];  /* storage for current/next/tendency/temp */
    WS_GRID *cur, *nxt, *tend, *tmp;
} WS_STATE;

static void WS_FN(grid_alloc)(WS_GRID* g, size_t n) {
    g->u = (WS_T*)calloc(n, sizeof(WS_T)); g->v = (WS_T*)calloc(n, sizeof(WS_T));
    g->h = (WS_T*)calloc(n, sizeof(WS_T)); g->p = (WS_T*)calloc(n, sizeof(WS_T));
    g->t = (WS_T*)calloc(n, sizeof(WS_T)); g->q = (WS_T*)calloc(n, sizeof(WS_T));
    g->vort = (WS_T*)calloc(n, sizeof(WS_T)); g->div = (WS_T*)calloc(n, sizeof(WS_T));
}

static void WS_FN(grid_free)(WS_GRID* g) {
    free(g->u); free(g->v); free(g->h); free(g->p); free(g->t); free(g->q); free(g->vort); free(g->div);
}

/* weather_grid.cpp:57-71 */
static void WS_FN(grid_reset)(WS_GRID* g, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        g->u[i] = (WS_T)0.0f; g->v[i] = (WS_T)0.0f; g->h[i] = (WS_T)10.0f;
        g->p[i] = (WS_T)1013.25f; g->t[i] = (WS_T)288.15f; g->q[i] = (WS_T)0.0f;
        g->vort[i] = (WS_T)0.0f; g->div[i] = (WS_T)0.0f;
    }
}

/* weather_grid.cpp:82-121: two serial passes */
void WS_FN(diagnostics)(const WS_T* u, const WS_T* v, WS_T* vort, WS_T* div, int W, int H, WS_T dx, WS_T dy) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const int l = x > 0 ? x - 1 : 0, r = x + 1 < W - 1 ? x + 1 : W - 1;
            const int t = y > 0 ? y - 1 : 0, b = y + 1 < H - 1 ? y + 1 : H - 1;
            const WS_T dv_dx = (v[(size_t)y * W + r] - v[(size_t)y * W + l]) / ((WS_T)2.0f * dx);
            const WS_T du_dy = (u[(size_t)b * W + x] - u[(size_t)t * W + x]) / ((WS_T)2.0f * dy);
            vort[(size_t)y * W + x] = dv_dx - du_dy;
        }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const int l = x > 0 ? x - 1 : 0, r = x + 1 < W - 1 ? x + 1 : W - 1;
            const int t = y > 0 ? y - 1 : 0, b = y + 1 < H - 1 ? y + 1 : H - 1;
            const WS_T du_dx = (u[(size_t)y * W + r] - u[(size_t)y * W + l]) / ((WS_T)2.0f * dx);
            const WS_T dv_dy = (v[(size_t)b * W + x] - v[(size_t)t * W + x]) / ((WS_T)2.0f * dy);
            div[(size_t)y * W + x] = du_dx + dv_dy;
        }
}

/* weather_simulation.cpp:473-540 (the OpenMP hot loop) */
void WS_FN(tendency)(const WS_T* U, const WS_T* V, const WS_T* Hh, WS_T* du, WS_T* dv, WS_T* dh,
                     int W, int H, WS_T dx, WS_T dy, WS_T gravity, WS_T coriolis_f) {
#pragma omp parallel for collapse(2)
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            const size_t idx = (size_t)y * W + x;
            const size_t il = x > 0 ? idx - 1 : idx;
            const size_t ir = x < W - 1 ? idx + 1 : idx;
            const size_t it = y > 0 ? idx - W : idx;
            const size_t ib = y < H - 1 ? idx + W : idx;
            const WS_T u = U[idx], v = V[idx], h = Hh[idx];
            const WS_T u_x = (U[ir] - U[il]) / ((WS_T)2.0f * dx);
            const WS_T u_y = (U[ib] - U[it]) / ((WS_T)2.0f * dy);
            const WS_T v_x = (V[ir] - V[il]) / ((WS_T)2.0f * dx);
            const WS_T v_y = (V[ib] - V[it]) / ((WS_T)2.0f * dy);
            const WS_T h_x = (Hh[ir] - Hh[il]) / ((WS_T)2.0f * dx);
            const WS_T h_y = (Hh[ib] - Hh[it]) / ((WS_T)2.0f * dy);
            du[idx] = -u * u_x - v * u_y - gravity * h_x + coriolis_f * v;
            dv[idx] = -u * v_x - v * v_y - gravity * h_y - coriolis_f * u;
            dh[idx] = -h * (u_x + v_y) - u * h_x - v * h_y;
        }
    }
}

WS_STATE* WS_FN(create)(int W, int H, int model, int method, double dx, double dy, double dt,
                        double g, double f, double max_time) {
    if (W <= 0 || H <= 0) return NULL;
    WS_STATE* s = (WS_STATE*)calloc(1, sizeof(WS_STATE));
    s->W = W; s->H = H; s->model = model; s->method = method;
    s->dx = (WS_T)dx; s->dy = (WS_T)dy; s->dt = (WS_T)dt; s->g = (WS_T)g; s->f = (WS_T)f;
    s->max_time = (WS_T)max_time;
    const size_t n = (size_t)W * H;
    for (int i = 0; i < 4; ++i) { WS_FN(grid_alloc)(&s->g_[i], n); WS_FN(grid_reset)(&s->g_[i], n); }
    s->cur = &s->g_[0]; s->nxt = &s->g_[1]; s->tend = &s->g_[2]; s->tmp = &s->g_[3];
    return s;
}

void WS_FN(destroy)(WS_STATE* s) {
    if (!s) return;
    for (int i = 0; i < 4; ++i) WS_FN(grid_free)(&s->g_[i]);
    free(s);
}

/* weather_simulation.cpp:46-66 (without the IC, which the caller writes via set_field) */
void WS_FN(initialize)(WS_STATE* s) {
    s->time = (WS_T)0.0; s->step = 0;
    WS_FN(grid_reset)(s->cur, (size_t)s->W * s->H);
}

static WS_T* WS_FN(field)(WS_GRID* g, int id) {
    switch (id) {
        case 0: return g->u; case 1: return g->v; case 2: return g->h; case 3: return g->p;
        case 4: return g->t; case 5: return g->q; case 6: return g->vort; case 7: return g->div;
    }
    return NULL;
}

void WS_FN(set_field)(WS_STATE* s, int id, const WS_T* src) {
    memcpy(WS_FN(field)(s->cur, id), src, sizeof(WS_T) * (size_t)s->W * s->H);
}
void WS_FN(get_field)(WS_STATE* s, int id, WS_T* dst) {
    memcpy(dst, WS_FN(field)(s->cur, id), sizeof(WS_T) * (size_t)s->W * s->H);
}
void WS_FN(calc_diagnostics)(WS_STATE* s) {
    WS_FN(diagnostics)(s->cur->u, s->cur->v, s->cur->vort, s->cur->div, s->W, s->H, s->dx, s->dy);
}
double WS_FN(get_time)(WS_STATE* s) { return (double)s->time; }
int WS_FN(get_step)(WS_STATE* s) { return s->step; }
void WS_FN(set_dt)(WS_STATE* s, double dt) { s->dt = (WS_T)dt; }

static void WS_FN(tend_of)(WS_STATE* s, WS_GRID* in) {
    WS_FN(tendency)(in->u, in->v, in->h, s->tend->u, s->tend->v, s->tend->h, s->W, s->H, s->dx, s->dy, s->g, s->f);
}

static void WS_FN(swap)(WS_STATE* s) { WS_GRID* t = s->cur; s->cur = s->nxt; s->nxt = t; }

/* :160-218 */
static void WS_FN(euler)(WS_STATE* s) {
    const size_t n = (size_t)s->W * s->H;
    const WS_T dt = s->dt;
    WS_FN(tend_of)(s, s->cur);
    for (size_t i = 0; i < n; ++i) {
        s->nxt->u[i] = s->cur->u[i] + dt * s->tend->u[i];
        s->nxt->v[i] = s->cur->v[i] + dt * s->tend->v[i];
    }
    for (size_t i = 0; i < n; ++i) s->nxt->h[i] = s->cur->h[i] + dt * s->tend->h[i];
    if (s->model == 2) {
        for (size_t i = 0; i < n; ++i) {
            s->nxt->t[i] = s->cur->t[i] + dt * s->tend->t[i];
            s->nxt->p[i] = s->cur->p[i] + dt * s->tend->p[i];
        }
    }
    WS_FN(swap)(s);
}

/* :220-323 */
static void WS_FN(rk2)(WS_STATE* s) {
    const size_t n = (size_t)s->W * s->H;
    const WS_T dt = s->dt;
    WS_FN(tend_of)(s, s->cur);
    for (size_t i = 0; i < n; ++i) {
        s->tmp->u[i] = s->cur->u[i] + (WS_T)0.5f * dt * s->tend->u[i];
        s->tmp->v[i] = s->cur->v[i] + (WS_T)0.5f * dt * s->tend->v[i];
    }
    for (size_t i = 0; i < n; ++i) s->tmp->h[i] = s->cur->h[i] + (WS_T)0.5f * dt * s->tend->h[i];
    if (s->model == 2) {
        for (size_t i = 0; i < n; ++i) {
            s->tmp->t[i] = s->cur->t[i] + (WS_T)0.5f * dt * s->tend->t[i];
            s->tmp->p[i] = s->cur->p[i] + (WS_T)0.5f * dt * s->tend->p[i];
        }
    }
    WS_FN(tend_of)(s, s->tmp);
    for (size_t i = 0; i < n; ++i) {
        s->nxt->u[i] = s->cur->u[i] + dt * s->tend->u[i];
        s->nxt->v[i] = s->cur->v[i] + dt * s->tend->v[i];
    }
    for (size_t i = 0; i < n; ++i) s->nxt->h[i] = s->cur->h[i] + dt * s->tend->h[i];
    if (s->model == 2) {
        for (size_t i = 0; i < n; ++i) {
            s->nxt->t[i] = s->cur->t[i] + dt * s->tend->t[i];
            s->nxt->p[i] = s->cur->p[i] + dt * s->tend->p[i];
        }
    }
    WS_FN(swap)(s);
}

/* :325-455 -- k1 is a reference into the tendency grid, overwritten by k2..k4 */
static void WS_FN(rk4)(WS_STATE* s) {
    if (s->model != 0) { WS_FN(rk2)(s); return; }
    const size_t n = (size_t)s->W * s->H;
    const WS_T dt = s->dt;
    WS_GRID *c = s->cur, *x = s->nxt, *tp = s->tmp, *k1 = s->tend;
    /* nine zero-initialised per-step vectors (:354-364) */
    WS_T *k2u = (WS_T*)calloc(n, sizeof(WS_T)), *k2v = (WS_T*)calloc(n, sizeof(WS_T)), *k2h = (WS_T*)calloc(n, sizeof(WS_T));
    WS_T *k3u = (WS_T*)calloc(n, sizeof(WS_T)), *k3v = (WS_T*)calloc(n, sizeof(WS_T)), *k3h = (WS_T*)calloc(n, sizeof(WS_T));
    WS_T *k4u = (WS_T*)calloc(n, sizeof(WS_T)), *k4v = (WS_T*)calloc(n, sizeof(WS_T)), *k4h = (WS_T*)calloc(n, sizeof(WS_T));
    WS_FN(tend_of)(s, c);
    for (size_t i = 0; i < n; ++i) { k2u[i] = k1->u[i]; k2v[i] = k1->v[i]; }
    for (size_t i = 0; i < n; ++i) k2h[i] = k1->h[i];
    for (size_t i = 0; i < n; ++i) {
        tp->u[i] = c->u[i] + (WS_T)0.5f * dt * k1->u[i];
        tp->v[i] = c->v[i] + (WS_T)0.5f * dt * k1->v[i];
    }
    for (size_t i = 0; i < n; ++i) tp->h[i] = c->h[i] + (WS_T)0.5f * dt * k1->h[i];
    WS_FN(tend_of)(s, tp);
    for (size_t i = 0; i < n; ++i) {
        k2u[i] = k1->u[i]; k2v[i] = k1->v[i];
        tp->u[i] = c->u[i] + (WS_T)0.5f * dt * k2u[i];
        tp->v[i] = c->v[i] + (WS_T)0.5f * dt * k2v[i];
    }
    for (size_t i = 0; i < n; ++i) { k2h[i] = k1->h[i]; tp->h[i] = c->h[i] + (WS_T)0.5f * dt * k2h[i]; }
    WS_FN(tend_of)(s, tp);
    for (size_t i = 0; i < n; ++i) {
        k3u[i] = k1->u[i]; k3v[i] = k1->v[i];
        tp->u[i] = c->u[i] + dt * k3u[i];
        tp->v[i] = c->v[i] + dt * k3v[i];
    }
    for (size_t i = 0; i < n; ++i) { k3h[i] = k1->h[i]; tp->h[i] = c->h[i] + dt * k3h[i]; }
    WS_FN(tend_of)(s, tp);
    for (size_t i = 0; i < n; ++i) { k4u[i] = k1->u[i]; k4v[i] = k1->v[i]; }
    for (size_t i = 0; i < n; ++i) k4h[i] = k1->h[i];
    for (size_t i = 0; i < n; ++i) {
        x->u[i] = c->u[i] + dt / (WS_T)6.0f * (k1->u[i] + (WS_T)2.0f * k2u[i] + (WS_T)2.0f * k3u[i] + k4u[i]);
        x->v[i] = c->v[i] + dt / (WS_T)6.0f * (k1->v[i] + (WS_T)2.0f * k2v[i] + (WS_T)2.0f * k3v[i] + k4v[i]);
    }
    for (size_t i = 0; i < n; ++i)
        x->h[i] = c->h[i] + dt / (WS_T)6.0f * (k1->h[i] + (WS_T)2.0f * k2h[i] + (WS_T)2.0f * k3h[i] + k4h[i]);
    free(k2u); free(k2v); free(k2h); free(k3u); free(k3v); free(k3h); free(k4u); free(k4v); free(k4h);
    WS_FN(swap)(s);
}

/* :117-158 */
void WS_FN(step)(WS_STATE* s) {
    switch (s->method) {
        case 1: WS_FN(rk2)(s); break;
        case 2: WS_FN(rk4)(s); break;
        default: WS_FN(euler)(s); break; /* Euler, AdamsBashforth, SemiImplicit, unknown */
    }
    s->time += s->dt;
    s->step++;
    WS_FN(calc_diagnostics)(s);
}

/* :68-103 -- returns the number of steps actually taken */
int WS_FN(run)(WS_STATE* s, int n) {
    int taken = 0;
    for (int i = 0; i < n; ++i) {
        WS_FN(step)(s);
        ++taken;
        if (s->time >= s->max_time) break;
    }
    return taken;
}

/* :105-115 */
int WS_FN(run_until)(WS_STATE* s, double max_time) {
    const WS_T mt = (WS_T)max_time;
    if (mt <= s->time) return 0;
    const int n = (int)((mt - s->time) / s->dt) + 1;
    return WS_FN(run)(s, n);
}

#undef WS_GRID
#undef WS_STATE
#undef WS_FN
#undef WS_CAT
#undef WS_CAT2
