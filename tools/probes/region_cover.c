/* region_cover.c -- diagnostic: which node pairs a frame's rays load, and what share of those loads an LDS
 * region of K pairs would serve if it held (a) the top levels (the product's depth cut), (b) the K pairs
 * with the largest parent boxes (a surface-area cut: closed upward, since a child's box lies in its parent's),
 * (c) the K most loaded pairs of this ray set (an oracle for a profile-guided region).
 * Closest-hit rays walk as the reference does (c1 first, culled against the running distance); shadow rays
 * stop at their first hit.  Plain fp32 (it counts loads; the kernels' exact arithmetic is not needed).
 * Input: u32 n_nodes, u32 n_tris, u32 n_rays; nodes (32-B std430); tris 9 f32; rays 8 f32 (o, d, tmax, kind
 * 0 closest / 1 shadow).  gcc -O2 -o /tmp/region_cover tools/probes/region_cover.c -lm  (region_cover.py) */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float mn[3]; uint32_t first; float mx[3]; uint32_t count; } Node;

static float box(const Node* n, const float* o, const float* inv) {
  float tn = -INFINITY, tf = INFINITY;
  for (int k = 0; k < 3; ++k) {
    float a = (n->mn[k] - o[k]) * inv[k], b = (n->mx[k] - o[k]) * inv[k];
    tn = fmaxf(tn, fminf(a, b));
    tf = fminf(tf, fmaxf(a, b));
  }
  if (tn > tf) return INFINITY;
  return tn >= 0.0f ? tn : tf;
}

static int tri(const float* v, const float* o, const float* d, float dist, float* tout) {
  float e1[3], e2[3], h[3], s[3], q[3];
  for (int k = 0; k < 3; ++k) e1[k] = v[3 + k] - v[k], e2[k] = v[6 + k] - v[k];
  h[0] = d[1] * e2[2] - d[2] * e2[1]; h[1] = d[2] * e2[0] - d[0] * e2[2]; h[2] = d[0] * e2[1] - d[1] * e2[0];
  float a = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
  if (a > -1e-4f && a < 1e-4f) return 0;
  float f = 1.0f / a;
  for (int k = 0; k < 3; ++k) s[k] = o[k] - v[k];
  float u = f * (s[0] * h[0] + s[1] * h[1] + s[2] * h[2]);
  if (u < 0.0f || u > 1.0f) return 0;
  q[0] = s[1] * e1[2] - s[2] * e1[1]; q[1] = s[2] * e1[0] - s[0] * e1[2]; q[2] = s[0] * e1[1] - s[1] * e1[0];
  float vv = f * (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]);
  if (vv < 0.0f || u + vv > 1.0f) return 0;
  float t = f * (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]);
  if (t > 1e-5f && t < dist) { *tout = t; return 1; }
  return 0;
}

static double* g_key;
static int cmp_desc(const void* a, const void* b) {
  double x = g_key[*(const uint32_t*)a], y = g_key[*(const uint32_t*)b];
  return x < y ? 1 : x > y ? -1 : 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* fp = fopen(argv[1], "rb");
  if (!fp) return 2;
  uint32_t hd[3];
  if (fread(hd, 4, 3, fp) != 3) return 2;
  const uint32_t nn = hd[0];
  Node* nodes = malloc(sizeof(Node) * nn);
  float* tris = malloc(sizeof(float) * 9 * (size_t)hd[1]);
  float* rays = malloc(sizeof(float) * 8 * (size_t)hd[2]);
  if (fread(nodes, sizeof(Node), nn, fp) != nn || fread(tris, 36, hd[1], fp) != hd[1] ||
      fread(rays, 32, hd[2], fp) != hd[2])
    return 2;
  fclose(fp);
  double* loads = calloc(nn, sizeof(double));  /* pair loads, keyed by the expanded (parent) node */
  int* depth = calloc(nn, sizeof(int));
  { /* depths */
    uint32_t* st = malloc(sizeof(uint32_t) * 2 * nn);
    int sp = 0;
    st[sp++] = 0;
    while (sp) {
      uint32_t i = st[--sp];
      if (nodes[i].count) continue;
      depth[nodes[i].first] = depth[nodes[i].first + 1] = depth[i] + 1;
      st[sp++] = nodes[i].first;
      st[sp++] = nodes[i].first + 1;
    }
    free(st);
  }
  double total = 0, kind_loads[2] = {0, 0};
  for (uint32_t r = 0; r < hd[2]; ++r) {
    const float* o = rays + 8 * (size_t)r;
    const float* d = o + 3;
    float dist = o[6];
    const int shadow = o[7] > 0.5f;
    float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
    uint32_t stk[256];
    int sp = 0, hit = 0;
    stk[sp++] = 0;
    while (sp > 0 && !(shadow && hit)) {
      const uint32_t ni = stk[--sp];
      const Node* n = &nodes[ni];
      float b = box(n, o, inv);
      if (!(b < dist) || isinf(b)) continue;
      if (n->count > 0) {
        for (uint32_t i = 0; i < n->count; ++i) {
          float t;
          if (tri(tris + 9 * (size_t)(n->first + i), o, d, dist, &t)) {
            dist = t;
            hit = 1;
            if (shadow) break;
          }
        }
        continue;
      }
      loads[ni] += 1;
      total += 1;
      kind_loads[shadow] += 1;
      if (sp < 254) {
        stk[sp++] = n->first;
        stk[sp++] = n->first + 1;
      }
    }
  }
  /* internal nodes reachable */
  uint32_t* ids = malloc(sizeof(uint32_t) * nn);
  uint32_t ni = 0;
  double* sa = calloc(nn, sizeof(double));
  for (uint32_t i = 0; i < nn; ++i)
    if (nodes[i].count == 0 && (i == 0 || depth[i] > 0)) {
      ids[ni++] = i;
      double dx = nodes[i].mx[0] - nodes[i].mn[0], dy = nodes[i].mx[1] - nodes[i].mn[1], dz = nodes[i].mx[2] - nodes[i].mn[2];
      sa[i] = dx * dy + dy * dz + dz * dx - 1e-9 * depth[i];  /* ties: shallower first */
    }
  printf("rays %u, pair loads %.0f (%.1f per ray; closest %.0f, shadow %.0f), internal nodes %u\n", hd[2], total,
         total / hd[2], kind_loads[0], kind_loads[1], ni);
  for (int dcut = 6; dcut <= 9; ++dcut) {
    double cov = 0;
    uint32_t k = 0;
    for (uint32_t j = 0; j < ni; ++j)
      if (depth[ids[j]] < dcut) cov += loads[ids[j]], ++k;
    printf("depth < %d: %u pairs, share of loads %.4f\n", dcut, k, cov / total);
  }
  const uint32_t Ks[] = {127, 160, 200, 255, 511};
  for (int m = 0; m < 2; ++m) {
    g_key = m == 0 ? sa : loads;
    qsort(ids, ni, sizeof(uint32_t), cmp_desc);
    for (size_t q = 0; q < sizeof(Ks) / sizeof(Ks[0]); ++q) {
      double cov = 0;
      for (uint32_t j = 0; j < Ks[q] && j < ni; ++j) cov += loads[ids[j]];
      printf("%s top %u: share of loads %.4f\n", m == 0 ? "surface-area cut" : "most-loaded pairs", Ks[q], cov / total);
    }
  }
  return 0;
}
