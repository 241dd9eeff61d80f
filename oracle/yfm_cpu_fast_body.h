/* yfm_cpu_fast_body.h — the per-step bodies of yfm_cpu_fast.c on 8-candidate vectors (GCC
 * vector extensions: every operation below acts on the 8 candidates of a block at once, which
 * the compiler lowers to AVX-512 or AVX2), instantiated once per state dimension M = FZ_M.
 * Included by yfm_cpu_fast.c only. */
#define M FZ_M

/* one collapsed-form step for the 8 candidates of a block; zt[j] = Z_j'ỹ_t */
static inline void FZ_NAME(collapsed_step)(block_t* s, const vd* zt, double ybar, double ytt, vl upd_mask,
                                           vl acc_mask) {
    vd ch[MMAX], c[MMAX], S[MMAX][MMAX], Lm[MMAX][MMAX], a[MMAX][MMAX], rd[MMAX];
    for (int i = 0; i < M; ++i) {
        vd x = vzero();
        for (int j = 1; j < M; ++j) x += s->R[i][j] * zt[j];
        ch[i] = x * s->rs2;
    }
    vd rr = vset(ytt);
    for (int j = 1; j < M; ++j) rr -= zt[j] * ch[j];
    ch[0] += ybar;
    for (int i = 0; i < M; ++i) {
        c[i] = ch[i] - s->beta[i];
        for (int j = 0; j <= i; ++j) S[i][j] = s->P[i][j] + s->R[i][j];
    }
    vd det = vset(1.0);
    for (int j = 0; j < M; ++j) { /* LDLᵀ of S = P + R */
        vd dj = S[j][j];
        for (int k = 0; k < j; ++k) dj -= a[j][k] * Lm[j][k];
        rd[j] = 1.0 / dj;
        det *= dj;
        for (int i = j + 1; i < M; ++i) {
            vd x = S[i][j];
            for (int k = 0; k < j; ++k) x -= a[i][k] * Lm[j][k];
            a[i][j] = x;
            Lm[i][j] = x * rd[j];
        }
    }
    /* x = S⁻¹c ; q = rr/σ² + c'x ; β_{t|t} = β + P x */
    vd x[MMAX];
    for (int i = 0; i < M; ++i) {
        vd y = c[i];
        for (int k = 0; k < i; ++k) y -= Lm[i][k] * x[k];
        x[i] = y;
    }
    for (int i = 0; i < M; ++i) x[i] *= rd[i];
    for (int i = M - 1; i >= 0; --i)
        for (int k = i + 1; k < M; ++k) x[i] -= Lm[k][i] * x[k];
    vd q = rr * s->rs2;
    for (int i = 0; i < M; ++i) q += c[i] * x[i];
    vd bf[MMAX], Pf[MMAX][MMAX];
    for (int i = 0; i < M; ++i) {
        vd y = s->beta[i];
        for (int k = 0; k < M; ++k) y += s->P[i][k] * x[k];
        bf[i] = y;
    }
    /* P_{t|t} = P S⁻¹ R, column by column */
    for (int j = 0; j < M; ++j) {
        vd xj[MMAX];
        for (int i = 0; i < M; ++i) {
            vd y = s->R[i][j];
            for (int k = 0; k < i; ++k) y -= Lm[i][k] * xj[k];
            xj[i] = y;
        }
        for (int i = 0; i < M; ++i) xj[i] *= rd[i];
        for (int i = M - 1; i >= 0; --i)
            for (int k = i + 1; k < M; ++k) xj[i] -= Lm[k][i] * xj[k];
        for (int i = 0; i <= j; ++i) {
            vd y = vzero();
            for (int k = 0; k < M; ++k) y += s->P[i][k] * xj[k];
            Pf[i][j] = y;
        }
    }
    /* β ← δ + Φβ_{t|t} ; P ← Φ P_{t|t} Φ' + Q */
    vd A[MMAX][MMAX];
    for (int i = 0; i < M; ++i) {
        vd y = s->delta[i];
        for (int j = 0; j < M; ++j) y += s->Phi[i][j] * bf[j];
        s->beta[i] = vsel(upd_mask, y, s->beta[i]);
        for (int j = 0; j < M; ++j) {
            vd z = vzero();
            for (int l = 0; l < M; ++l) z += s->Phi[i][l] * (l <= j ? Pf[l][j] : Pf[j][l]);
            A[i][j] = z;
        }
    }
    for (int i = 0; i < M; ++i)
        for (int j = i; j < M; ++j) {
            vd z = s->Q[i][j];
            for (int l = 0; l < M; ++l) z += A[i][l] * s->Phi[j][l];
            s->P[i][j] = vsel(upd_mask, z, s->P[i][j]);
            s->P[j][i] = s->P[i][j];
        }
    s->last_det = vsel(upd_mask, det, s->last_det);
    s->last_q = vsel(upd_mask, q, s->last_q);
    const vl add = upd_mask & acc_mask;
    s->mant *= vsel(add, vabs(det), vset(1.0));
    s->sumq += vsel(add, q, vzero());
    s->neg |= add & (det < 0.0);
}

/* the prediction-only step of a NaN column (filter.jl:126-140): stale F and v re-added */
static void FZ_NAME(predict_block)(block_t* s, vl upd_mask, vl acc_mask) {
    vd A[MMAX][MMAX], nb[MMAX];
    for (int i = 0; i < M; ++i) {
        vd y = s->delta[i];
        for (int j = 0; j < M; ++j) y += s->Phi[i][j] * s->beta[j];
        nb[i] = y;
        for (int j = 0; j < M; ++j) {
            vd z = vzero();
            for (int l = 0; l < M; ++l) z += s->Phi[i][l] * s->P[l][j];
            A[i][j] = z;
        }
    }
    for (int i = 0; i < M; ++i) {
        s->beta[i] = vsel(upd_mask, nb[i], s->beta[i]);
        for (int j = i; j < M; ++j) {
            vd z = s->Q[i][j];
            for (int l = 0; l < M; ++l) z += A[i][l] * s->Phi[j][l];
            s->P[i][j] = vsel(upd_mask, z, s->P[i][j]);
            s->P[j][i] = s->P[i][j];
        }
    }
    const vl add = upd_mask & acc_mask;
    s->mant *= vsel(add, vabs(s->last_det), vset(1.0));
    s->sumq += vsel(add, s->last_q, vzero());
    s->neg |= add & (s->last_det < 0.0);
}
#undef M
