/*
 * lbm_oracle.c -- TEST INFRASTRUCTURE ONLY (see lbm_oracle.h for the contract).
 *
 * Serial C restatement of the reference CUDA kernels and host set-up code.  Every
 * function cites the reference lines it restates.  Compile with -ffp-contract=off:
 * the reference's fp32 expression trees (and its single fp64 sub-expression in
 * feq[14]) are reproduced literally, because a 1e-6 relative-L2 match is below the
 * FMA-contraction floor (finding 5).
 */
#include "lbm_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* D3Q19 as implied by the reference pull offsets (ldc.cu:76-182): fnq[q] <- cell - e_q */
static const int EX[19] = {0, 1, -1, 0, 0, 0, 0, 1, 1, -1, -1, 1, 1, -1, -1, 0, 0, 0, 0};
static const int EY[19] = {0, 0, 0, 1, -1, 0, 0, 1, -1, 1, -1, 0, 0, 0, 0, 1, -1, 1, -1};
static const int EZ[19] = {0, 0, 0, 0, 0, 1, -1, 0, 0, 0, 0, 1, -1, 1, -1, 1, 1, -1, -1};
/* opposite directions, from the bounce-back swap ldc.cu:184-201 */
static const int OPP[19] = {0, 2, 1, 4, 3, 6, 5, 10, 9, 8, 7, 14, 13, 12, 11, 18, 17, 16, 15};

struct orc_lbm {
    int kind, nx, ny, nz, ldc_order;
    long ncell;
    float tau;
    int8_t* geo;
    float *src, *dst;                /* d_scr / d_dst */
    float *rho, *ux, *uy, *uz;       /* d_rho ... (zero-initialised like fresh device memory) */
    float *inlet_uy, *outlet_uy;     /* nx*nz tables (POISEUILLE: kernel uygt; MASK: bc.txt) */
    long bad_reads;
    int steps;
    orc_bc bcs[16];                  /* ORC_GENERIC (tables owned) */
    int nbc;
    float sum_current;               /* ldc.cu:652 sum_current */
    int residual_mode;               /* ORC_SUM_*: how S is summed (orc_set_residual_mode) */
    int cub_ipt, cub_vec, cub_grid;  /* ORC_SUM_CUB_TREE: items per thread, vector width, grid cap */
    float* terms;                    /* ORC_SUM_CUB_TREE: the |u| terms in reference storage order */
};

static inline long cidx(const orc_lbm* o, int x, int y, int z) {
    return (long)x + (long)o->nx * ((long)y + (long)o->ny * (long)z);
}

/* ------------------------------------------------------------------------- */
/* geometry                                                                  */
/* ------------------------------------------------------------------------- */

/* ldc.cu:468-502 -- ghost 0, wall 1, fluid 3, lid 2 (y = ny-2 plane) */
void orc_geo_ldc(int nx, int ny, int nz, int8_t* geo) {
    long n = (long)nx * ny * nz;
    memset(geo, 0, (size_t)n);
    for (int z = 1; z < nz - 1; z++)
        for (int y = 1; y < ny - 1; y++)
            for (int x = 1; x < nx - 1; x++) geo[x + (long)nx * (y + (long)ny * z)] = 1;
    for (int x = 2; x < nx - 2; x++)
        for (int y = 2; y < ny - 2; y++)
            for (int z = 2; z < nz - 2; z++) geo[x + (long)nx * (y + (long)ny * z)] = 3;
    int y = ny - 2;
    for (int x = 1; x < nx - 1; x++)
        for (int z = 1; z < nz - 1; z++) geo[x + (long)nx * (y + (long)ny * z)] = 2;
}

static int imin(int a, int b) { return a < b ? a : b; }

/* 18-neighbour ghost marking (Poiseulle.cu:138-254, bifurcation.cu:122-239): every
 * geo==0 neighbour (q=1..18) of a cell for which `is_src(code)` holds becomes -1. */
static void mark_ghosts(int nx, int ny, int nz, int8_t* geo, int poiseuille_rule) {
    for (int z = 1; z < nz - 1; z++)
        for (int y = 1; y < ny - 1; y++)
            for (int x = 1; x < nx - 1; x++) {
                int g = geo[x + (long)nx * (y + (long)ny * z)];
                int src = poiseuille_rule ? (g == 1 || g == 2 || g == 3) : (g == 1);
                if (!src) continue;
                for (int q = 1; q < 19; q++) {
                    long c2 = (x + EX[q]) + (long)nx * ((y + EY[q]) + (long)ny * (z + EZ[q]));
                    if (geo[c2] == 0) geo[c2] = -1;
                }
            }
}

/* Poiseulle.cu:52-255: pipe along y, radius (nx-1)/2 */
void orc_geo_poiseuille(int nx, int ny, int nz, int8_t* geo) {
    long n = (long)nx * ny * nz;
    int8_t* flag = (int8_t*)calloc((size_t)n, 1);
    int* g = (int*)calloc((size_t)n, sizeof(int));
    float radius = (nx - 1) / 2.0f;
    float center_x = (nx - 1) / 2.0f, center_z = (nz - 1) / 2.0f;
#define F(x, y, z) flag[(x) + (long)nx * ((y) + (long)ny * (z))]
#define G(x, y, z) g[(x) + (long)nx * ((y) + (long)ny * (z))]
    /* to binary matrix (80-91) */
    for (int x = 0; x < nx; x++)
        for (int y = 1; y < ny - 1; y++)
            for (int z = 0; z < nz; z++) {
                float dist = sqrtf(powf(x - center_x, 2) + powf(z - center_z, 2));
                if (dist <= radius) { F(x, y, z) = 1; G(x, y, z) = 1; }
            }
    /* distance transform, fluid = 4 (93-108): three passes over the unchanged flag */
    for (int t = 0; t < 3; t++)
        for (int x = 1; x < nx - 1; x++)
            for (int y = 2; y < ny - 2; y++)
                for (int z = 1; z < nz - 1; z++) {
                    int minx = imin(F(x + 1, y, z), F(x - 1, y, z));
                    int miny = imin(F(x, y - 1, z), F(x, y + 1, z));
                    int minz = imin(F(x, y, z - 1), F(x, y, z + 1));
                    G(x, y, z) += imin(imin(minx, miny), minz);
                }
    /* left end = 2 (110-120) */
    {
        int y = 1;
        for (int x = 1; x < nx - 1; x++)
            for (int z = 1; z < nz - 1; z++)
                G(x, y, z) += imin(imin(F(x + 1, y, z), F(x - 1, y, z)), imin(F(x, y, z - 1), F(x, y, z + 1)));
    }
    /* right end = 3 (122-134): two passes */
    {
        int y = ny - 2;
        for (int t = 0; t < 2; t++)
            for (int x = 1; x < nx - 1; x++)
                for (int z = 1; z < nz - 1; z++)
                    G(x, y, z) += imin(imin(F(x + 1, y, z), F(x - 1, y, z)), imin(F(x, y, z - 1), F(x, y, z + 1)));
    }
#undef F
#undef G
    for (long c = 0; c < n; c++) geo[c] = (int8_t)g[c];
    mark_ghosts(nx, ny, nz, geo, 1); /* 138-254: around geo 1,2,3 */
    free(flag);
    free(g);
}

/* bifurcation.cu:50-60: whitespace-separated ints, loop z, y, x (x fastest) */
int orc_read_geo_txt(const char* path, int n, int32_t* raw) {
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    int i = 0, v;
    while (i < n && fscanf(f, "%d ", &v) == 1) raw[i++] = v;
    fclose(f);
    return i;
}

/* bifurcation.cu:36-253 */
void orc_geo_mask(int nx, int ny, int nz, const int32_t* raw, int8_t* geo) {
    long n = (long)nx * ny * nz;
    int* g = (int*)calloc((size_t)n, sizeof(int));
    for (long c = 0; c < n; c++) g[c] = raw[c]; /* h_geo = flag = raw */
#define F(x, y, z) raw[(x) + (long)nx * ((y) + (long)ny * (z))]
#define G(x, y, z) g[(x) + (long)nx * ((y) + (long)ny * (z))]
    /* 63-72: zero the y=0 and y=ny-1 planes (h_geo only) */
    for (int x = 1; x < nx - 1; x++)
        for (int z = 1; z < nz - 1; z++) { G(x, 0, z) = 0; G(x, ny - 1, z) = 0; }
    /* 75-90: fluid = 4 */
    for (int t = 0; t < 3; t++)
        for (int x = 1; x < nx - 1; x++)
            for (int y = 2; y < ny - 2; y++)
                for (int z = 1; z < nz - 1; z++) {
                    int minx = imin(F(x + 1, y, z), F(x - 1, y, z));
                    int miny = imin(F(x, y - 1, z), F(x, y + 1, z));
                    int minz = imin(F(x, y, z - 1), F(x, y, z + 1));
                    G(x, y, z) += imin(imin(minx, miny), minz);
                }
    /* 92-103: inlet = 2 copied from the y=2 class */
    for (int x = 1; x < nx - 1; x++)
        for (int z = 1; z < nz - 1; z++) {
            int v = 0;
            if (G(x, 2, z) == 1) v = 1;
            if (G(x, 2, z) == 4) v = 2;
            G(x, 1, z) = v;
        }
    /* 105-118: outlet = 3 copied from the y=ny-3 class (loop runs twice; idempotent) */
    for (int t = 0; t < 2; t++)
        for (int x = 1; x < nx - 1; x++)
            for (int z = 1; z < nz - 1; z++) {
                int v = 0;
                if (G(x, ny - 3, z) == 1) v = 1;
                if (G(x, ny - 3, z) == 4) v = 3;
                G(x, ny - 2, z) = v;
            }
#undef F
#undef G
    for (long c = 0; c < n; c++) geo[c] = (int8_t)g[c];
    mark_ghosts(nx, ny, nz, geo, 0); /* 122-239: around geo == 1 only */
    free(g);
}

/* coronary.cu:45-56: the same token stream, loop z, x, y (y fastest) */
int orc_read_geo_txt_zxy(const char* path, int nx, int ny, int nz, int32_t* raw) {
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    int i = 0, v;
    for (int z = 0; z < nz; z++)
        for (int x = 0; x < nx; x++)
            for (int y = 0; y < ny; y++) {
                if (fscanf(f, "%d ", &v) != 1) { fclose(f); return i; }
                raw[x + (long)nx * (y + (long)ny * z)] = v;
                i++;
            }
    fclose(f);
    return i;
}

/* coronary.cu:31-275 (geo_pre).  The reference hard-codes five end planes for its
 * 291 x 291 x 372 box (75-143); here each end is ends[7 e .. 7 e + 6] =
 * {axis (0 = x plane, 2 = z plane), plane, lo0, hi0, lo1, hi1, passes}, looped as the
 * reference loops them: x planes over y in [lo0, hi0) outer, z in [lo1, hi1) inner, with the
 * y and z neighbours (75-99); z planes over [lo0, hi0) x [lo1, hi1) with the y and x
 * neighbours (101-143). */
void orc_geo_coronary(int nx, int ny, int nz, const int32_t* raw, int n_ends, const int* ends, int8_t* geo) {
    long n = (long)nx * ny * nz;
    int* g = (int*)calloc((size_t)n, sizeof(int));
    for (long c = 0; c < n; c++) g[c] = raw[c]; /* 45-56: h_geo = flag = tmp */
#define F(x, y, z) raw[(x) + (long)nx * ((y) + (long)ny * (z))]
#define G(x, y, z) g[(x) + (long)nx * ((y) + (long)ny * (z))]
    /* 58-73: distance transform, fluid = 4 */
    for (int t = 0; t < 3; t++)
        for (int x = 1; x < nx - 1; x++)
            for (int y = 1; y < ny - 1; y++)
                for (int z = 1; z < nz - 1; z++) {
                    int minx = imin(F(x + 1, y, z), F(x - 1, y, z));
                    int miny = imin(F(x, y - 1, z), F(x, y + 1, z));
                    int minz = imin(F(x, y, z - 1), F(x, y, z + 1));
                    G(x, y, z) = G(x, y, z) + imin(imin(minx, miny), minz);
                }
    for (int e = 0; e < n_ends; e++) {
        const int* E = ends + 7 * e;
        for (int t = 0; t < E[6]; t++) {
            if (E[0] == 0) { /* 75-99: x = plane, y outer, z inner */
                int x = E[1];
                for (int y = E[2]; y < E[3]; y++)
                    for (int z = E[4]; z < E[5]; z++) {
                        int miny = imin(F(x, y - 1, z), F(x, y + 1, z));
                        int minz = imin(F(x, y, z - 1), F(x, y, z + 1));
                        G(x, y, z) = G(x, y, z) + imin(miny, minz);
                    }
            } else { /* 101-143: z = plane; the window's first range is x, the second y */
                int z = E[1];
                for (int x = E[2]; x < E[3]; x++)
                    for (int y = E[4]; y < E[5]; y++) {
                        int miny = imin(F(x, y - 1, z), F(x, y + 1, z));
                        int minz = imin(F(x - 1, y, z), F(x + 1, y, z)); /* the reference's name */
                        G(x, y, z) = G(x, y, z) + imin(miny, minz);
                    }
            }
        }
    }
#undef F
#undef G
    for (long c = 0; c < n; c++) geo[c] = (int8_t)g[c];
    mark_ghosts(nx, ny, nz, geo, 0); /* 145-260: around geo == 1 */
    free(g);
}

/* bifurcation.cu:294-325 */
int orc_read_bc_txt(const char* path, int nx, int ny, int nz, const int8_t* geo, int skip_blocks,
                    float* inlet_uy, float* outlet_uy) {
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    int ntok = 0;
    float tmp;
    for (int s = 0; s < skip_blocks * nx * nz; s++) {
        if (fscanf(f, "%f ", &tmp) != 1) { fclose(f); return ntok; }
        ntok++;
    }
    int y = 1;
    for (int z = 0; z < nz; z++)
        for (int x = 0; x < nx; x++) {
            if (fscanf(f, "%f ", &tmp) != 1) tmp = 0.0f; else ntok++;
            inlet_uy[x + z * nx] = (geo[x + (long)nx * (y + (long)ny * z)] == 2) ? tmp : 0.0f;
        }
    y = ny - 2;
    for (int z = 0; z < nz; z++)
        for (int x = 0; x < nx; x++) {
            if (fscanf(f, "%f ", &tmp) != 1) tmp = 0.0f; else ntok++;
            outlet_uy[x + z * nx] = (geo[x + (long)nx * (y + (long)ny * z)] == 3) ? tmp : 0.0f;
        }
    fclose(f);
    return ntok;
}

/* Poiseulle.cu:257-271 */
int orc_index_transform(int nx, int ny, int nz, const int8_t* geo, int32_t* index) {
    int n = 0;
    for (int z = 0; z < nz; z++)
        for (int y = 0; y < ny; y++)
            for (int x = 0; x < nx; x++) {
                long c = x + (long)nx * (y + (long)ny * z);
                index[c] = geo[c] != 0 ? n++ : -1;
            }
    return n;
}

/* ------------------------------------------------------------------------- */
/* equilibria                                                                */
/* ------------------------------------------------------------------------- */

/* the update-kernel form, ldc.cu:330-348 (== Poiseulle.cu:543-561, bifurcation.cu:587-624).
 * feq[14] carries the reference's fp64 literal "3.0*tmp_uz*tmp_uz" (ldc.cu:344). */
static void feq_update(float tmp_rho, float tmp_ux, float tmp_uy, float tmp_uz, float* feq) {
    feq[0] = tmp_rho/3.0f * (1.0f - 1.5f*tmp_ux*tmp_ux -1.5f* tmp_uy*tmp_uy -1.5f* tmp_uz*tmp_uz);
    feq[1] = tmp_rho /18.0f * (1.0f + 3.0f* tmp_ux + 3.0f*tmp_ux*tmp_ux -1.5f* tmp_uy*tmp_uy -1.5f* tmp_uz*tmp_uz);
    feq[2] = tmp_rho /18.0f * (1.0f - 3.0f* tmp_ux + 3.0f*tmp_ux*tmp_ux -1.5f* tmp_uy*tmp_uy -1.5f* tmp_uz*tmp_uz);
    feq[3] = tmp_rho /18.0f * (1.0f + 3.0f* tmp_uy + 3.0f*tmp_uy*tmp_uy - 1.5f*tmp_ux*tmp_ux -1.5f* tmp_uz*tmp_uz);
    feq[4] = tmp_rho /18.0f * (1.0f - 3.0f* tmp_uy + 3.0f*tmp_uy*tmp_uy - 1.5f*tmp_ux*tmp_ux -1.5f* tmp_uz*tmp_uz);
    feq[5] = tmp_rho /18.0f * (1.0f + 3.0f* tmp_uz + 3.0f*tmp_uz*tmp_uz - 1.5f*tmp_ux*tmp_ux -1.5f* tmp_uy*tmp_uy);
    feq[6] = tmp_rho /18.0f* (1.0f - 3.0f* tmp_uz + 3.0f*tmp_uz*tmp_uz - 1.5f*tmp_ux*tmp_ux -1.5f* tmp_uy*tmp_uy);
    feq[7] = tmp_rho /36.0f* (1.0f + 3.0f* (tmp_ux + tmp_uy) + 3.0f*tmp_ux*tmp_ux + 3.0f*tmp_uy*tmp_uy + 9.0f*tmp_ux*tmp_uy -1.5f* tmp_uz*tmp_uz);
    feq[8] = tmp_rho /36.0f * (1.0f + 3.0f* (tmp_ux - tmp_uy) + 3.0f*tmp_ux*tmp_ux + 3.0f*tmp_uy*tmp_uy - 9.0f*tmp_ux*tmp_uy-1.5f* tmp_uz*tmp_uz);
    feq[9] = tmp_rho /36.0f * (1.0f + 3.0f* (tmp_uy - tmp_ux) + 3.0f* tmp_ux*tmp_ux + 3.0f*tmp_uy*tmp_uy - 9.0f*tmp_ux*tmp_uy-1.5f* tmp_uz*tmp_uz);
    feq[10] = tmp_rho /36.0f * (1.0f - 3.0f* (tmp_ux + tmp_uy) + 3.0f*tmp_ux*tmp_ux + 3.0f*tmp_uy*tmp_uy + 9.0f*tmp_ux*tmp_uy-1.5f* tmp_uz*tmp_uz);
    feq[11] = tmp_rho /36.0f * (1.0f + 3.0f* (tmp_ux + tmp_uz) + 3.0f* tmp_ux*tmp_ux + 3.0f*tmp_uz*tmp_uz + 9.0f*tmp_ux*tmp_uz-1.5f* tmp_uy*tmp_uy);
    feq[12] = tmp_rho /36.0f* (1.0f + 3.0f* (tmp_ux - tmp_uz) + 3.0f* tmp_ux*tmp_ux + 3.0f*tmp_uz*tmp_uz - 9.0f*tmp_ux*tmp_uz-1.5f* tmp_uy*tmp_uy);
    feq[13] = tmp_rho /36.0f * (1.0f + 3.0f* (tmp_uz - tmp_ux) + 3.0f* tmp_ux*tmp_ux + 3.0f*tmp_uz*tmp_uz - 9.0f*tmp_ux*tmp_uz-1.5f* tmp_uy*tmp_uy);
    feq[14] = tmp_rho /36.0f * (1.0f - 3.0f* (tmp_ux + tmp_uz) + 3.0f* tmp_ux*tmp_ux + 3.0*tmp_uz*tmp_uz + 9.0f*tmp_ux*tmp_uz -1.5f* tmp_uy*tmp_uy);
    feq[15] = tmp_rho /36.0f * (1.0f + 3.0f* (tmp_uy + tmp_uz) + 3.0f* tmp_uy*tmp_uy + 3.0f*tmp_uz*tmp_uz + 9.0f*tmp_uy*tmp_uz- 1.5f*tmp_ux*tmp_ux);
    feq[16] = tmp_rho /36.0f * (1.0f + 3.0f* (tmp_uz - tmp_uy) + 3.0f* tmp_uy*tmp_uy + 3.0f*tmp_uz*tmp_uz - 9.0f*tmp_uy*tmp_uz - 1.5f*tmp_ux*tmp_ux);
    feq[17] = tmp_rho /36.0f * (1.0f + 3.0f* (tmp_uy - tmp_uz) + 3.0f* tmp_uy*tmp_uy + 3.0f*tmp_uz*tmp_uz - 9.0f*tmp_uy*tmp_uz - 1.5f*tmp_ux*tmp_ux);
    feq[18] = tmp_rho /36.0f * (1.0f - 3.0f* (tmp_uy + tmp_uz) + 3.0f* tmp_uy*tmp_uy + 3.0f*tmp_uz*tmp_uz + 9.0f*tmp_uy*tmp_uz - 1.5f*tmp_ux*tmp_ux);
}

/* boundary-value equilibrium: the reference's NEE "tmp" terms are fp32 throughout; they equal
 * feq_update for every q they use except q = 14 on a z face (coronary.cu:870-871), where the
 * fp64 sub-expression of the update form is absent */
static void feq_bc(float tmp_rho, float tmp_ux, float tmp_uy, float tmp_uz, float* feq) {
    feq_update(tmp_rho, tmp_ux, tmp_uy, tmp_uz, feq);
    feq[14] = tmp_rho /36.0f * (1.0f - 3.0f* (tmp_ux + tmp_uz) + 3.0f* tmp_ux*tmp_ux + 3.0f*tmp_uz*tmp_uz + 9.0f*tmp_ux*tmp_uz -1.5f* tmp_uy*tmp_uy);
}

/* the LDC initialize() form, ldc.cu:542-571 */
static void feq_init_ldc(float tmp_rho, float tmp_ux, float tmp_uy, float tmp_uz, float* feq) {
    static const float wi[19] = { 1.0f / 3.0f, 1.0f / 18.0f,1.0f / 18.0f,1.0f / 18.0f,1.0f / 18.0f,1.0f / 18.0f,1.0f / 18.0f,1.0f / 36.0f,1.0f / 36.0f,1.0f / 36.0f,1.0f / 36.0f,1.0f / 36.0f,1.0f / 36.0f,1.0f / 36.0f,1.0f / 36.0f,1.0f / 36.0f,1.0f / 36.0f,1.0f / 36.0f,1.0f / 36.0f };
    float ux2 = tmp_ux*tmp_ux, uy2 = tmp_uy*tmp_uy, uz2 = tmp_uz*tmp_uz;
    float uxyz2 = ux2 + uy2 + uz2, uxy2 = ux2 + uy2, uxz2 = ux2 + uz2, uyz2 = uy2 + uz2;
    float uxy = 2.0f*tmp_ux*tmp_uy, uxz = 2.0f*tmp_ux*tmp_uz, uyz = 2.0f*tmp_uy*tmp_uz;
    feq[0] = tmp_rho * wi[0] * (1.0f - 1.5f*uxyz2);
    feq[1] = tmp_rho * wi[1] * (1.0f + 3.0f* tmp_ux + 4.5f*ux2 - 1.5f*uxyz2);
    feq[2] = tmp_rho * wi[2] * (1.0f - 3.0f* tmp_ux + 4.5f*ux2 - 1.5f*uxyz2);
    feq[3] = tmp_rho * wi[3] * (1.0f + 3.0f* tmp_uy + 4.5f*uy2 - 1.5f*uxyz2);
    feq[4] = tmp_rho * wi[4] * (1.0f - 3.0f* tmp_uy + 4.5f*uy2 - 1.5f*uxyz2);
    feq[5] = tmp_rho * wi[5] * (1.0f + 3.0f* tmp_uz + 4.5f*uz2 - 1.5f*uxyz2);
    feq[6] = tmp_rho * wi[6] * (1.0f - 3.0f* tmp_uz + 4.5f*uz2 - 1.5f*uxyz2);
    feq[7] = tmp_rho * wi[7] * (1.0f + 3.0f* (tmp_ux + tmp_uy) + 4.5f* (uxy2 + uxy) - 1.5f*uxyz2);
    feq[8] = tmp_rho * wi[8] * (1.0f + 3.0f* (tmp_ux - tmp_uy) + 4.5f* (uxy2 - uxy) - 1.5f* uxyz2);
    feq[9] = tmp_rho * wi[9] * (1.0f + 3.0f* (tmp_uy - tmp_ux) + 4.5f* (uxy2 - uxy) - 1.5f* uxyz2);
    feq[10] = tmp_rho * wi[10] * (1.0f - 3.0f* (tmp_ux + tmp_uy) + 4.5f* (uxy2 + uxy) - 1.5f* uxyz2);
    feq[11] = tmp_rho * wi[11] * (1.0f + 3.0f* (tmp_ux + tmp_uz) + 4.5f* (uxz2 + uxz) - 1.5f* uxyz2);
    feq[12] = tmp_rho * wi[12] * (1.0f + 3.0f* (tmp_ux - tmp_uz) + 4.5f* (uxz2 - uxz) - 1.5f* uxyz2);
    feq[13] = tmp_rho * wi[13] * (1.0f + 3.0f* (tmp_uz - tmp_ux) + 4.5f* (uxz2 - uxz) - 1.5f* uxyz2);
    feq[14] = tmp_rho * wi[14] * (1.0f - 3.0f* (tmp_ux + tmp_uz) + 4.5f* (uxz2 + uxz) - 1.5f* uxyz2);
    feq[15] = tmp_rho * wi[15] * (1.0f + 3.0f* (tmp_uy + tmp_uz) + 4.5f* (uyz2 + uyz) - 1.5f* uxyz2);
    feq[16] = tmp_rho * wi[16] * (1.0f + 3.0f* (tmp_uz - tmp_uy) + 4.5f* (uyz2 - uyz) - 1.5f* uxyz2);
    feq[17] = tmp_rho * wi[17] * (1.0f + 3.0f* (tmp_uy - tmp_uz) + 4.5f* (uyz2 - uyz) - 1.5f* uxyz2);
    feq[18] = tmp_rho * wi[18] * (1.0f - 3.0f* (tmp_uy + tmp_uz) + 4.5f* (uyz2 + uyz) - 1.5f* uxyz2);
}

/* ------------------------------------------------------------------------- */
/* solver                                                                    */
/* ------------------------------------------------------------------------- */

orc_lbm* orc_create(int kind, int nx, int ny, int nz, const int8_t* geo, float tau, int ldc_order,
                    const float* inlet_uy, const float* outlet_uy) {
    orc_lbm* o = (orc_lbm*)calloc(1, sizeof(orc_lbm));
    o->kind = kind; o->nx = nx; o->ny = ny; o->nz = nz; o->tau = tau; o->ldc_order = ldc_order;
    o->ncell = (long)nx * ny * nz;
    o->geo = (int8_t*)malloc((size_t)o->ncell);
    memcpy(o->geo, geo, (size_t)o->ncell);
    o->src = (float*)calloc((size_t)o->ncell * 19, sizeof(float));
    o->dst = (float*)calloc((size_t)o->ncell * 19, sizeof(float));
    o->rho = (float*)calloc((size_t)o->ncell, sizeof(float));
    o->ux = (float*)calloc((size_t)o->ncell, sizeof(float));
    o->uy = (float*)calloc((size_t)o->ncell, sizeof(float));
    o->uz = (float*)calloc((size_t)o->ncell, sizeof(float));
    o->inlet_uy = (float*)calloc((size_t)nx * nz, sizeof(float));
    o->outlet_uy = (float*)calloc((size_t)nx * nz, sizeof(float));
    if (kind == ORC_POISEUILLE) {
        /* Poiseulle.cu:590,597: the kernel's parabola with the hard-coded u_max */
        float u_max = 0.09714700668f;
        for (int k = 0; k < nz; k++)
            for (int i = 0; i < nx; i++) {
                float uygt = u_max*(1.0f-(powf(i-(nx - 1) / 2.0f,2.f)+powf(k-(nz - 1) / 2.0f,2.f))/powf((nx - 1) / 2.0f,2.f));
                o->inlet_uy[i + k * nx] = uygt;
                o->outlet_uy[i + k * nx] = uygt;
            }
    } else if (kind == ORC_MASK) {
        if (inlet_uy) memcpy(o->inlet_uy, inlet_uy, sizeof(float) * nx * nz);
        if (outlet_uy) memcpy(o->outlet_uy, outlet_uy, sizeof(float) * nx * nz);
    }
    return o;
}

orc_lbm* orc_create_generic(int nx, int ny, int nz, const int8_t* geo, float tau, const orc_bc* bcs, int nbc) {
    if (nbc < 0 || nbc > 16) return NULL;
    orc_lbm* o = orc_create(ORC_GENERIC, nx, ny, nz, geo, tau, ORC_LDC_TWO_PHASE, NULL, NULL);
    o->nbc = nbc;
    for (int k = 0; k < nbc; k++) {
        o->bcs[k] = bcs[k];
        if (bcs[k].table) {
            int axis = bcs[k].face >> 1;
            long nt = axis == 0 ? (long)ny * nz : axis == 1 ? (long)nx * nz : (long)nx * ny;
            float* t = (float*)malloc(sizeof(float) * (size_t)nt);
            memcpy(t, bcs[k].table, sizeof(float) * (size_t)nt);
            o->bcs[k].table = t;
        }
    }
    return o;
}

void orc_feq(float rho, float ux, float uy, float uz, float* feq19) { feq_update(rho, ux, uy, uz, feq19); }
void orc_feq_bc(float rho, float ux, float uy, float uz, float* feq19) { feq_bc(rho, ux, uy, uz, feq19); }

/* the boundary velocity of code entry b at cell (x,y,z) */
static void bc_velocity(const orc_lbm* o, const orc_bc* b, int x, int y, int z, float* u) {
    u[0] = b->u[0]; u[1] = b->u[1]; u[2] = b->u[2];
    if (b->table) {
        int axis = b->face >> 1;
        long ti = axis == 0 ? y + (long)z * o->ny : axis == 1 ? x + (long)z * o->nx : x + (long)y * o->nx;
        u[axis] = b->table[ti];
    }
}

static const orc_bc* find_bc(const orc_lbm* o, int code) {
    for (int k = 0; k < o->nbc; k++)
        if (o->bcs[k].code == code) return &o->bcs[k];
    return NULL;
}

/* generic NEE cell (coronary.cu:716-944 generalised) */
static void nee_generic_cell(orc_lbm* o, const orc_bc* b, int x, int y, int z) {
    const long n = o->ncell;
    const long c = cidx(o, x, y, z);
    const float tau = o->tau;
    const int axis = b->face >> 1, sgn = (b->face & 1) ? -1 : 1;
    float ubc[3];
    bc_velocity(o, b, x, y, z, ubc);
    for (int q = 1; q < 19; q++) {
        int e = axis == 0 ? EX[q] : axis == 1 ? EY[q] : EZ[q];
        if (e != sgn) continue;
        int x2 = x + EX[q], y2 = y + EY[q], z2 = z + EZ[q];
        if (x2 < 0 || y2 < 0 || z2 < 0 || x2 >= o->nx || y2 >= o->ny || z2 >= o->nz) continue;
        long c2 = cidx(o, x2, y2, z2);
        float tmp_rho = o->rho[c2], tmp_ux = o->ux[c2], tmp_uy = o->uy[c2], tmp_uz = o->uz[c2];
        float feq[19], ebc[19];
        feq_update(tmp_rho, tmp_ux, tmp_uy, tmp_uz, feq);
        if (b->kind == 2) feq_bc(b->rho, tmp_ux, tmp_uy, tmp_uz, ebc);
        else feq_bc(b->kind == 1 ? b->rho : tmp_rho, ubc[0], ubc[1], ubc[2], ebc);
        o->dst[q * n + c] = ebc[q] + (o->dst[q * n + c2] - feq[q])*(1.0f - 1.0f / tau);
    }
}

void orc_destroy(orc_lbm* o) {
    if (!o) return;
    for (int k = 0; k < o->nbc; k++) free((void*)o->bcs[k].table);
    free(o->geo); free(o->src); free(o->dst);
    free(o->rho); free(o->ux); free(o->uy); free(o->uz);
    free(o->inlet_uy); free(o->outlet_uy); free(o->terms);
    free(o);
}

void orc_initialize(orc_lbm* o) {
    const int nx = o->nx, ny = o->ny, nz = o->nz;
    const long n = o->ncell;
    float feq[19];
    if (o->kind == ORC_LDC) {
        /* ldc.cu:504-580 -- every cell, rho=1, u=0; uz = u_max on y = ny-1 and ny-2 */
        const float C_U = 2.4705f;
        float u_max = 0.15f / C_U;
        for (int z = 0; z < nz; z++)
            for (int y = 0; y < ny; y++)
                for (int x = 0; x < nx; x++) {
                    long c = cidx(o, x, y, z);
                    float uz = (y == ny - 1 || y == ny - 2) ? u_max : 0.0f;
                    feq_init_ldc(1.0f, 0.0f, 0.0f, uz, feq);
                    for (int q = 0; q < 19; q++) o->src[q * n + c] = o->dst[q * n + c] = feq[q];
                }
    } else if (o->kind == ORC_GENERIC) {
        /* coronary.cu:280-330 generalised: stored cells at rest, velocity-boundary cells at u_bc */
        for (int z = 0; z < nz; z++)
            for (int y = 0; y < ny; y++)
                for (int x = 0; x < nx; x++) {
                    long c = cidx(o, x, y, z);
                    if (o->geo[c] == 0) continue;
                    float u[3] = {0.0f, 0.0f, 0.0f};
                    const orc_bc* b = find_bc(o, o->geo[c]);
                    if (b && b->kind != 2) bc_velocity(o, b, x, y, z, u);
                    feq_update(1.0f, u[0], u[1], u[2], feq);
                    for (int q = 0; q < 19; q++) o->src[q * n + c] = o->dst[q * n + c] = feq[q];
                }
    } else {
        /* Poiseulle.cu:273-382 / bifurcation.cu:329-427 -- stored cells only (index >= 0) */
        const float C_U = 1.5441f;
        float u_max = 0.15f / C_U; /* Poiseulle.cu:44 */
        float center_x = (nx - 1) / 2.0f, center_z = (nz - 1) / 2.0f, radius = (nx - 1) / 2.0f;
        for (int z = 0; z < nz; z++)
            for (int y = 0; y < ny; y++)
                for (int x = 0; x < nx; x++) {
                    long c = cidx(o, x, y, z);
                    if (o->geo[c] == 0) continue;
                    float ux = 0.0f, uy = 0.0f, uz = 0.0f;
                    if (o->kind == ORC_POISEUILLE) {
                        if (y == 0 || y == 1 || y == ny - 1 || y == ny - 2)
                            uy = u_max*(1.0f-(powf(x-center_x,2)+powf(z-center_z,2))/powf(radius,2));
                    } else {
                        if (y == 1) uy = o->inlet_uy[x + z * nx];
                        if (y == ny - 2) uy = o->outlet_uy[x + z * nx];
                    }
                    feq_update(1.0f, ux, uy, uz, feq);
                    for (int q = 0; q < 19; q++) o->src[q * n + c] = o->dst[q * n + c] = feq[q];
                }
    }
    o->steps = 0;
    o->sum_current = 0.0f;
    memset(o->rho, 0, sizeof(float) * n); memset(o->ux, 0, sizeof(float) * n);
    memset(o->uy, 0, sizeof(float) * n); memset(o->uz, 0, sizeof(float) * n);
}

/* coronary.cu:277-350 (initialize) for a generic instance holding the coronary codes: every
 * stored cell rho = 1, u = 0; code 2 u_x = 0.1745f/C_U, 3 u_x = 0.1f/C_U, 5/6/7 u_z = 0.02f/C_U
 * (float quotients; the boundary kernel's are double, coronary.cu:717, 797), then the update-form
 * equilibrium (309-348, the same expression trees as feq_update). */
void orc_initialize_coronary(orc_lbm* o) {
    const long n = o->ncell;
    const float C_U = 2.74909090909091f;
    float feq[19];
    for (long c = 0; c < n; c++) {
        int g = o->geo[c];
        if (g == 0) continue;
        float ux = 0.0f, uy = 0.0f, uz = 0.0f;
        if (g == 2) ux = 0.1745f / C_U;
        if (g == 3) ux = 0.1f / C_U;
        if (g == 5) uz = 0.02f / C_U;
        if (g == 6) uz = 0.02f / C_U;
        if (g == 7) uz = 0.02f / C_U;
        feq_update(1.0f, ux, uy, uz, feq);
        for (int q = 0; q < 19; q++) o->src[q * n + c] = o->dst[q * n + c] = feq[q];
    }
}

static int fluid_code(const orc_lbm* o) { return o->kind == ORC_LDC ? 3 : 4; }

/* One fluid-cell update (ldc.cu:204-368 / Poiseulle.cu:398-581 / bifurcation.cu:444-635). */
static long update_cell(orc_lbm* o, int x, int y, int z) {
    const long n = o->ncell;
    const long c = cidx(o, x, y, z);
    const float tau = o->tau;
    float fnq[19], feq[19];
    long bad = 0;
    for (int q = 0; q < 19; q++) {
        long c2 = cidx(o, x - EX[q], y - EY[q], z - EZ[q]);
        if (o->kind != ORC_LDC && o->geo[c2] == 0) bad++; /* index -1 in the reference */
        fnq[q] = o->src[q * n + c2];
    }
    float tmp_rho = 0.f;
    for (int k = 0; k < 19; k++) tmp_rho = tmp_rho + fnq[k];
    float tmp_ux = (fnq[1] - fnq[2] + fnq[7] + fnq[8] - fnq[9] - fnq[10] + fnq[11] + fnq[12] - fnq[13] - fnq[14]) / tmp_rho;
    float tmp_uy = (fnq[3] - fnq[4] + fnq[7] - fnq[8] + fnq[9] - fnq[10] + fnq[15] - fnq[16] + fnq[17] - fnq[18]) / tmp_rho;
    float tmp_uz = (fnq[5] - fnq[6] + fnq[11] - fnq[12] + fnq[13] - fnq[14] + fnq[15] + fnq[16] - fnq[17] - fnq[18]) / tmp_rho;
    o->ux[c] = tmp_ux; o->uy[c] = tmp_uy; o->uz[c] = tmp_uz; o->rho[c] = tmp_rho;
    feq_update(tmp_rho, tmp_ux, tmp_uy, tmp_uz, feq);
    for (int q = 0; q < 19; q++) o->dst[q * n + c] = fnq[q] - (fnq[q] - feq[q]) / tau;
    return bad;
}

/* the update kernel over every cell of class `code` (cells are independent: the
 * pass reads only src and writes only dst/macros of its own cell) */
static void update_pass(orc_lbm* o, int code) {
    const int nx = o->nx, ny = o->ny, nz = o->nz;
    long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
    for (int z = 0; z < nz; z++)
        for (int y = 0; y < ny; y++)
            for (int x = 0; x < nx; x++)
                if (o->geo[cidx(o, x, y, z)] == code) bad += update_cell(o, x, y, z);
    o->bad_reads += bad;
}

/* LDC wall branch, in place on d_scr (ldc.cu:75-202) */
static void ldc_wall_cell(orc_lbm* o, int x, int y, int z) {
    const long n = o->ncell;
    const long c = cidx(o, x, y, z);
    float fnq[19];
    for (int q = 1; q < 19; q++) fnq[q] = o->src[q * n + cidx(o, x - EX[q], y - EY[q], z - EZ[q])];
    for (int q = 1; q < 19; q++) o->src[q * n + c] = fnq[OPP[q]];
}

/* Wall half-way bounce-back on d_dst after the update (Poiseulle.cu:601-746,
 * bifurcation.cu:654-799), with the kernels' y wrap. */
static void post_wall_cell(orc_lbm* o, int x, int y, int z) {
    const long n = o->ncell;
    const long c = cidx(o, x, y, z);
    float fnq[19];
    for (int q = 1; q < 19; q++) {
        int xx = x - EX[q], yy = (y - EY[q] + o->ny) % o->ny, zz = z - EZ[q];
        if (xx < 0 || xx >= o->nx || zz < 0 || zz >= o->nz) { fnq[q] = 0.0f; continue; }
        fnq[q] = o->dst[q * n + cidx(o, xx, yy, zz)];
    }
    for (int q = 1; q < 19; q++) o->dst[q * n + c] = fnq[OPP[q]];
}

/* LDC lid, ldc.cu:391-456 -- hand-simplified tmp terms kept literally */
static void ldc_lid_cell(orc_lbm* o, int x, int y, int z) {
    const long n = o->ncell;
    const long c = cidx(o, x, y, z);
    const float tau = o->tau;
    const float C_U = 2.4705f;
    float u_max = 0.15f / C_U;
    static const int S[5] = {4, 8, 10, 16, 18};
    for (int s = 0; s < 5; s++) {
        int q = S[s];
        long c2 = cidx(o, x + EX[q], y + EY[q], z + EZ[q]);
        float tmp_rho = o->rho[c2], tmp_ux = o->ux[c2], tmp_uy = o->uy[c2], tmp_uz = o->uz[c2];
        float feq[19], tmp;
        feq_update(tmp_rho, tmp_ux, tmp_uy, tmp_uz, feq);
        switch (q) {
            case 4: tmp = tmp_rho/18.0f* (1.0f - 1.5f*u_max*u_max); break;
            case 8: tmp = tmp_rho/36.0f  * (1.0f - 1.5f* u_max*u_max); break;
            case 10: tmp = tmp_rho /36.0f  * (1.0f - 1.5f* u_max*u_max); break;
            case 16: tmp = tmp_rho /36.0f * (1.0f + 3.0f*u_max + 3.0f*u_max*u_max); break;
            default: tmp = tmp_rho /36.0f * (1.0f - 3.0f*u_max + 3.0f*u_max*u_max); break;
        }
        o->dst[q * n + c] = tmp + (o->dst[q * n + c2] - feq[q])*(1.0f - 1.0f / tau);
    }
}

/* Velocity NEE with a (0,uygt,0) profile: Poiseuille inlet/outlet (Poiseulle.cu:748-891),
 * bifurcation inlet (bifurcation.cu:950-1021). sign=+1: inlet set {3,7,9,15,17};
 * sign=-1: outlet set {4,8,10,16,18}. */
static void nee_velocity_cell(orc_lbm* o, int x, int y, int z, int sign, float uygt) {
    const long n = o->ncell;
    const long c = cidx(o, x, y, z);
    const float tau = o->tau;
    static const int SIN[5] = {3, 7, 9, 15, 17}, SOUT[5] = {4, 8, 10, 16, 18};
    for (int s = 0; s < 5; s++) {
        int q = sign > 0 ? SIN[s] : SOUT[s];
        long c2 = cidx(o, x + EX[q], y + EY[q], z + EZ[q]);
        float tmp_rho = o->rho[c2], tmp_ux = o->ux[c2], tmp_uy = o->uy[c2], tmp_uz = o->uz[c2];
        float feq[19], tmp;
        feq_update(tmp_rho, tmp_ux, tmp_uy, tmp_uz, feq);
        float W = (q == 3 || q == 4) ? 18.0f : 36.0f;
        if (sign > 0) tmp = tmp_rho / W * (1.0f + 3.0f* uygt + 3.0f*uygt*uygt);
        else          tmp = tmp_rho / W * (1.0f - 3.0f* uygt + 3.0f*uygt*uygt);
        o->dst[q * n + c] = tmp + (o->dst[q * n + c2] - feq[q])*(1.0f - 1.0f / tau);
    }
}

/* bifurcation pressure outlet, rho=1, u = u_nb (bifurcation.cu:877-948) */
static void nee_pressure_cell(orc_lbm* o, int x, int y, int z) {
    const long n = o->ncell;
    const long c = cidx(o, x, y, z);
    const float tau = o->tau;
    static const int S[5] = {4, 8, 10, 16, 18};
    for (int s = 0; s < 5; s++) {
        int q = S[s];
        long c2 = cidx(o, x + EX[q], y + EY[q], z + EZ[q]);
        float tmp_rho = o->rho[c2], tmp_ux = o->ux[c2], tmp_uy = o->uy[c2], tmp_uz = o->uz[c2];
        float feq[19], one[19];
        feq_update(tmp_rho, tmp_ux, tmp_uy, tmp_uz, feq);
        /* tmp = 1.f/W * (same polynomial): feq with rho = 1 has the identical tree */
        feq_update(1.0f, tmp_ux, tmp_uy, tmp_uz, one);
        o->dst[q * n + c] = one[q] + (o->dst[q * n + c2] - feq[q])*(1.0f - 1.0f / tau);
    }
}

/* calc_vel_square's terms (ldc.cu:460-466) in the reference storage order: LDC brick order
 * over the brick-padded box (8x8x8, ldc.cu:71), otherwise the compact z,y,x order of
 * index_transform (Poiseulle.cu:257-271).  Cells never written hold 0.  Returns the count. */
static long velsum_terms(const orc_lbm* o, float* t) {
    const int nx = o->nx, ny = o->ny, nz = o->nz;
    long n = 0;
    if (o->kind == ORC_LDC) {
        int bx = 1 + (nx - 1) / 8, by = 1 + (ny - 1) / 8, bz = 1 + (nz - 1) / 8;
        for (int b = 0; b < bx * by * bz; b++) {
            int ix = b % bx, iy = (b / bx) % by, iz = b / (bx * by);
            for (int k = 0; k < 8; k++)
                for (int j = 0; j < 8; j++)
                    for (int i = 0; i < 8; i++) {
                        int x = ix * 8 + i, y = iy * 8 + j, z = iz * 8 + k;
                        float v = 0.f;
                        if (x < nx && y < ny && z < nz) {
                            long c = cidx(o, x, y, z);
                            float ux = o->ux[c], uy = o->uy[c], uz = o->uz[c];
                            v = sqrtf(ux * ux + uy * uy + uz * uz);
                        }
                        t[n++] = v;
                    }
        }
    } else {
        for (long c = 0; c < o->ncell; c++) {
            if (o->geo[c] == 0) continue;
            float ux = o->ux[c], uy = o->uy[c], uz = o->uz[c];
            t[n++] = sqrtf(ux * ux + uy * uy + uz * uz);
        }
    }
    return n;
}

/* CUB-style device reduction of n fp32 terms (cub::DeviceReduce / thrust::reduce's two-pass
 * scheme, restated from CUB's published algorithm; the reference's CUDA/CUB version and GPU
 * fix its parameters, which it does not record, so they are arguments):
 *  pass 1: grid = min(tiles, grid_cap) blocks of 256 threads over tiles of 256*ipt items,
 *          "even share" (block b takes a contiguous run of tiles, the first tiles % grid
 *          blocks one tile more).  In a full tile thread t loads vec-wide vectors at
 *          4t + 256*vec*i (i < ipt/vec) and folds the ipt items serially into its running
 *          sum (the first tile starts the sum with its first item); a partial tile is read
 *          striped (t, t + 256, ...).  Block reduction: 32-lane warps reduce by shuffle-down
 *          trees (offsets 1, 2, 4, 8, 16; lane l adds lane l + offset when that lane holds
 *          data), then thread 0 adds the warp sums serially.
 *  pass 2: one block over the grid partials (one per thread, striped), reduced the same way;
 *          S = 0.f + that (thrust's init). */
static float warp_tree(float* v, int valid) {   /* v[0..32): lane values; valid lanes hold data */
    for (int off = 1; off < 32; off <<= 1)
        for (int l = 0; l < 32; l++)             /* shuffle-down: reads of the previous round */
            if (l + off < valid && (l % (2 * off)) == 0) v[l] = v[l + off] + v[l];
    return v[0];
}
static float block_reduce(float* agg, int num_valid) {
    float lane[32], s = 0.f;
    for (int w = 0; w < 8; w++) {
        int valid = num_valid - 32 * w;
        if (valid <= 0) break;
        if (valid > 32) valid = 32;
        for (int l = 0; l < 32; l++) lane[l] = agg[32 * w + l];
        float ws = warp_tree(lane, valid);
        s = (w == 0) ? ws : s + ws;
    }
    return s;
}
float orc_cub_reduce(const float* v, long n, int ipt, int vec, int grid_cap) {
    const long tile = 256L * ipt;
    const long tiles = (n + tile - 1) / tile;
    if (n <= 0) return 0.f;
    long grid = tiles < grid_cap ? tiles : grid_cap;
    if (tiles <= 1) grid = 1;
    const long avg = tiles / grid, big = tiles - avg * grid;
    float* part = (float*)malloc(sizeof(float) * (size_t)grid);
    float agg[256];
    for (long b = 0; b < grid; b++) {
        long t0 = b < big ? b * (avg + 1) : big * (avg + 1) + (b - big) * avg;
        long off = t0 * tile, end = off + (avg + (b < big)) * tile;
        if (end > n) end = n;
        int first = 1, num_valid = 256;
        for (; off + tile <= end; off += tile, first = 0)
            for (int t = 0; t < 256; t++) {
                float s = first ? 0.f : agg[t];
                int k0 = first;
                if (first) s = v[off + (long)vec * t];
                for (int i = 0; i < ipt / vec; i++)
                    for (int k = 0; k < vec; k++) {
                        if (k0) { k0 = 0; continue; }
                        s = s + v[off + (long)vec * t + 256L * vec * i + k];
                    }
                agg[t] = s;
            }
        if (off < end) {  /* partial tile: striped */
            long valid = end - off;
            for (int t = 0; t < 256; t++) {
                long i = t;
                if (first) {
                    if (i >= valid) continue;
                    agg[t] = v[off + i];
                    i += 256;
                }
                for (; i < valid; i += 256) agg[t] = agg[t] + v[off + i];
            }
            if (first) num_valid = valid < 256 ? (int)valid : 256;
        }
        part[b] = block_reduce(agg, num_valid);
    }
    float s;
    if (grid == 1) s = part[0];
    else {  /* pass 2: one partial tile of grid items */
        long i;
        for (int t = 0; t < 256; t++) {
            i = t;
            if (i >= grid) continue;
            agg[t] = part[i];
            for (i += 256; i < grid; i += 256) agg[t] = agg[t] + part[i];
        }
        s = block_reduce(agg, grid < 256 ? (int)grid : 256);
    }
    free(part);
    return 0.f + s;
}

/* thrust::reduce of calc_vel_square (ldc.cu:460-466, 660-662): by default emulated serially
 * in fp32 over the reference storage order (velsum_terms) */
float orc_velsum(const orc_lbm* o) {
    if (o->residual_mode == ORC_SUM_CUB_TREE) {
        long n = velsum_terms(o, o->terms);
        return orc_cub_reduce(o->terms, n, o->cub_ipt, o->cub_vec, o->cub_grid);
    }
    if (o->residual_mode == ORC_SUM_FP64) {
        /* liblbm's S: the same fp32 |u| terms accumulated in fp64 over the stored cells (the
         * off-fluid ones hold 0), rounded to fp32 once -- an accurate summation, the limit
         * thrust's fp32 tree approaches; the reference's own order is unspecified */
        double d = 0.0;
        for (long c = 0; c < o->ncell; c++) {
            if (o->kind != ORC_LDC && o->geo[c] == 0) continue;
            float ux = o->ux[c], uy = o->uy[c], uz = o->uz[c];
            d += (double)sqrtf(ux * ux + uy * uy + uz * uz);
        }
        return (float)d;
    }
    float s = 0.f;
    const int nx = o->nx, ny = o->ny, nz = o->nz;
    if (o->kind == ORC_LDC) {
        int bx = 1 + (nx - 1) / 8, by = 1 + (ny - 1) / 8, bz = 1 + (nz - 1) / 8;
        for (int b = 0; b < bx * by * bz; b++) {
            int ix = b % bx, iy = (b / bx) % by, iz = b / (bx * by);
            for (int k = 0; k < 8; k++)
                for (int j = 0; j < 8; j++)
                    for (int i = 0; i < 8; i++) {
                        int x = ix * 8 + i, y = iy * 8 + j, z = iz * 8 + k;
                        if (x >= nx || y >= ny || z >= nz) continue;
                        long c = cidx(o, x, y, z);
                        float ux = o->ux[c], uy = o->uy[c], uz = o->uz[c];
                        /* powf(u, 2.f) of ldc.cu:464; gcc folds it to u*u (verified equal) */
                        s = s + sqrtf(ux * ux + uy * uy + uz * uz);
                    }
        }
    } else {
        for (long c = 0; c < o->ncell; c++) {
            if (o->geo[c] == 0) continue;
            float ux = o->ux[c], uy = o->uy[c], uz = o->uz[c];
            s = s + sqrtf(ux * ux + uy * uy + uz * uz);
        }
    }
    return s;
}

static void swap_buffers(orc_lbm* o) { float* t = o->src; o->src = o->dst; o->dst = t; }

static void step_once(orc_lbm* o) {
    const int nx = o->nx, ny = o->ny, nz = o->nz;
    const int fc = fluid_code(o);
    if (o->kind == ORC_LDC) {
        if (o->ldc_order == ORC_LDC_SERIAL_EMU) {
            /* emulation order of the racy in-place update: blocks z,y,x; threads y,x; koff 7..0 */
            int bx = 1 + (nx - 1) / 8, by = 1 + (ny - 1) / 8, bz = 1 + (nz - 1) / 8;
            for (int kb = 0; kb < bz; kb++)
                for (int jb = 0; jb < by; jb++)
                    for (int ib = 0; ib < bx; ib++)
                        for (int ty = 0; ty < 8; ty++)
                            for (int tx = 0; tx < 8; tx++)
                                for (int koff = 7; koff >= 0; koff--) {
                                    int x = ib * 8 + tx, y = jb * 8 + ty, z = kb * 8 + koff;
                                    if (x >= nx || y >= ny || z >= nz) continue;
                                    int g = o->geo[cidx(o, x, y, z)];
                                    if (g == 1) ldc_wall_cell(o, x, y, z);
                                    if (g == 3) o->bad_reads += update_cell(o, x, y, z);
                                }
        } else {
            /* two-phase (race-free) semantics: every wall write before every fluid read */
            for (int z = 0; z < nz; z++)
                for (int y = 0; y < ny; y++)
                    for (int x = 0; x < nx; x++)
                        if (o->geo[cidx(o, x, y, z)] == 1) ldc_wall_cell(o, x, y, z);
            update_pass(o, 3);
        }
        for (int z = 0; z < nz; z++)
            for (int y = 0; y < ny; y++)
                for (int x = 0; x < nx; x++)
                    if (o->geo[cidx(o, x, y, z)] == 2) ldc_lid_cell(o, x, y, z);
    } else if (o->kind == ORC_GENERIC) {
        update_pass(o, 4);
        for (int z = 0; z < nz; z++)
            for (int y = 0; y < ny; y++)
                for (int x = 0; x < nx; x++)
                    if (o->geo[cidx(o, x, y, z)] == 1) post_wall_cell(o, x, y, z);
        for (int z = 0; z < nz; z++)
            for (int y = 0; y < ny; y++)
                for (int x = 0; x < nx; x++) {
                    const orc_bc* b = find_bc(o, o->geo[cidx(o, x, y, z)]);
                    if (b) nee_generic_cell(o, b, x, y, z);
                }
    } else {
        update_pass(o, fc);
        for (int z = 0; z < nz; z++)
            for (int y = 0; y < ny; y++)
                for (int x = 0; x < nx; x++)
                    if (o->geo[cidx(o, x, y, z)] == 1) post_wall_cell(o, x, y, z);
        for (int z = 0; z < nz; z++)
            for (int y = 0; y < ny; y++)
                for (int x = 0; x < nx; x++) {
                    int g = o->geo[cidx(o, x, y, z)];
                    if (g == 3) {
                        if (o->kind == ORC_POISEUILLE) nee_velocity_cell(o, x, y, z, -1, o->outlet_uy[x + z * nx]);
                        else nee_pressure_cell(o, x, y, z);
                    } else if (g == 2) {
                        nee_velocity_cell(o, x, y, z, +1, o->inlet_uy[x + z * nx]);
                    }
                }
    }
    swap_buffers(o); /* ldc.cu:664-666 */
    o->steps++;
}

void orc_step(orc_lbm* o, int nsteps, float* residual_hist) {
    for (int s = 0; s < nsteps; s++) {
        step_once(o);
        float sum_next = orc_velsum(o);
        float residual = fabsf(sum_next - o->sum_current) / sum_next; /* ldc.cu:668 */
        if (residual_hist) residual_hist[s] = residual;
        o->sum_current = sum_next;
    }
}

/* ldc.cu:653-685 / Poiseulle.cu:986-1019 */
int orc_run_converge(orc_lbm* o, int max_it, int stag_max, float tol, float* last_residual) {
    int k = 0, tol_count = 0;
    float residual = 0.0f;
    while (k <= max_it && tol_count <= stag_max) {
        step_once(o);
        float sum_next = orc_velsum(o);
        residual = fabsf(sum_next - o->sum_current) / sum_next;
        k++;
        o->sum_current = sum_next;
        if (residual <= tol) tol_count++;
    }
    if (last_residual) *last_residual = residual;
    return k;
}

int orc_steps_done(const orc_lbm* o) { return o->steps; }

void orc_get_macros(const orc_lbm* o, float* rho, float* ux, float* uy, float* uz) {
    size_t b = sizeof(float) * (size_t)o->ncell;
    if (rho) memcpy(rho, o->rho, b);
    if (ux) memcpy(ux, o->ux, b);
    if (uy) memcpy(uy, o->uy, b);
    if (uz) memcpy(uz, o->uz, b);
}

void orc_get_f(const orc_lbm* o, float* f) { memcpy(f, o->src, sizeof(float) * 19 * (size_t)o->ncell); }

void orc_set_f(orc_lbm* o, const float* f) {
    memcpy(o->src, f, sizeof(float) * 19 * (size_t)o->ncell);
    memcpy(o->dst, f, sizeof(float) * 19 * (size_t)o->ncell);
}

long orc_bad_reads(const orc_lbm* o) { return o->bad_reads; }

void orc_set_residual_fp64(orc_lbm* o, int on) { o->residual_mode = on ? ORC_SUM_FP64 : ORC_SUM_SERIAL; }

int orc_set_residual_mode(orc_lbm* o, int mode, int ipt, int vec, int grid_cap) {
    if (mode < ORC_SUM_SERIAL || mode > ORC_SUM_CUB_TREE) return -1;
    if (mode == ORC_SUM_CUB_TREE) {
        if (ipt < 1 || vec < 1 || ipt % vec || grid_cap < 1) return -1;
        if (!o->terms) {
            long cap = o->ncell + 8L * 8 * 8 * (o->nx / 8 + 2) * (o->ny / 8 + 2) * 2;  /* brick padding */
            if (o->kind == ORC_LDC) {
                long bx = 1 + (o->nx - 1) / 8, by = 1 + (o->ny - 1) / 8, bz = 1 + (o->nz - 1) / 8;
                cap = bx * by * bz * 512;
            }
            o->terms = (float*)malloc(sizeof(float) * (size_t)cap);
            if (!o->terms) return -1;
        }
        o->cub_ipt = ipt; o->cub_vec = vec; o->cub_grid = grid_cap;
    }
    o->residual_mode = mode;
    return 0;
}

/* bifurcation.cu:1158-1175 */
double orc_calc_res_bif(const orc_lbm* o) {
    long double sum1 = 0.0L;
    for (int z = 1; z < o->nz - 1; z++)
        for (int y = 2; y < o->ny - 2; y++)
            for (int x = 1; x < o->nx - 1; x++) {
                long c = cidx(o, x, y, z);
                if (o->geo[c] >= 4) {
                    float vtmp = powf(o->ux[c], 2.f) + powf(o->uy[c], 2.f) + powf(o->uz[c], 2.f);
                    sum1 = sum1 + vtmp;
                }
            }
    return (double)sum1;
}
