/* shadow_steps.c -- diagnostic: memory round trips (fused sub-steps) a shadow ray takes in global-scene mode,
 * under the kernel's schedule and under schedules that use a shadow ray's freedom of visit order.
 *
 * A fused sub-step (traversal.hpp trav_fused) issues one set of loads per lane and then tests what they
 * returned: at an internal node its child pair, plus -- when the right child c1 is internal -- c1's child
 * pair, which the layout places next (the right-spine step expands both levels); at a leaf its next two
 * triangles.  Then the lane pops if nothing is current.  A shadow ray only needs CheckHit(...).hit, so it
 * may expand nodes in any order:
 *   schedule 0: the kernel's (reference order, spine step);
 *   schedule 1: as 0, and when the spine slot is free (c1 is a leaf) the step also expands the stack's top
 *               entry if it is internal (its pair in the spine's registers), pushing what that adds;
 *   schedule 2: as 1, and a leaf step whose leaf has one triangle left also expands an internal stack top
 *               (3 + 4 float4 of loads, within the step's 8).
 * Input: the binary of tools/probes/shadow_order.py.  Output: mean sub-steps, node pairs and triangle tests per ray.
 *   gcc -O2 -o /tmp/shadow_steps tools/probes/shadow_steps.c -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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

static int tri(const float* v, const float* o, const float* d, float dist) {
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
  return t > 1e-5f && t < dist;
}

typedef struct { uint32_t ref, cnt; } Ent;  /* internal: ref = node index, cnt = 0; leaf: first tri, count */

static const Node* g_nodes;
static const float* g_tris;
static double g_pairs, g_tests;
static unsigned char* g_depth;       /* depth of each node (root 0) */
static double g_pairs_by_depth[64];  /* node pairs expanded, by the depth of the expanded node (schedule 0) */
static int g_sched;

/* Expands internal node `n`: the children that pass go to *cur (c1 first) and the stack. */
static void expand(uint32_t n, const float* o, const float* inv, float dist, Ent* cur, int* has, Ent* stk, int* sp) {
  g_pairs += 1;
  if (g_sched == 0) g_pairs_by_depth[g_depth[n] < 63 ? g_depth[n] : 63] += 1;
  const uint32_t c0 = g_nodes[n].first, c1 = c0 + 1;
  const int v0 = box(&g_nodes[c0], o, inv) < dist, v1 = box(&g_nodes[c1], o, inv) < dist;
  Ent e0 = {g_nodes[c0].count ? g_nodes[c0].first : c0, g_nodes[c0].count};
  Ent e1 = {g_nodes[c1].count ? g_nodes[c1].first : c1, g_nodes[c1].count};
  if (v0 && v1) stk[(*sp)++] = e0;
  if (v1) *cur = e1, *has = 1;
  else if (v0) *cur = e0, *has = 1;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* fp = fopen(argv[1], "rb");
  if (!fp) return 2;
  uint32_t hd[3];
  if (fread(hd, 4, 3, fp) != 3) return 2;
  Node* nodes = malloc(sizeof(Node) * hd[0]);
  float* tris = malloc(sizeof(float) * 9 * (size_t)hd[1]);
  float* rays = malloc(sizeof(float) * 7 * (size_t)hd[2]);
  if (fread(nodes, sizeof(Node), hd[0], fp) != hd[0] || fread(tris, 36, hd[1], fp) != hd[1] ||
      fread(rays, 28, hd[2], fp) != hd[2])
    return 2;
  fclose(fp);
  g_nodes = nodes;
  g_tris = tris;
  g_depth = calloc(hd[0], 1);
  for (uint32_t i = 0; i < hd[0]; ++i)  /* children follow their parent in the array's pair order: one pass */
    if (nodes[i].count == 0 && nodes[i].first + 1 < hd[0])
      g_depth[nodes[i].first] = g_depth[nodes[i].first + 1] = (unsigned char)(g_depth[i] + 1);
  for (int sched = 0; sched < 3; ++sched) {
    g_sched = sched;
    double steps = 0;
    long occl = 0;
    g_pairs = g_tests = 0;
    for (uint32_t r = 0; r < hd[2]; ++r) {
      const float* o = rays + 7 * (size_t)r;
      const float* d = o + 3;
      const float dist = o[6];
      float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
      Ent stk[256];
      int sp = 0, has = 0, hit = 0;
      Ent cur = {0, 0};
      g_pairs += 1;  /* the root box (tested when the ray starts) */
      if (box(&nodes[0], o, inv) < dist) {
        cur.ref = nodes[0].count ? nodes[0].first : 0;
        cur.cnt = nodes[0].count;
        has = 1;
      }
      while (has && !hit) {
        steps += 1;
        Ent next = {0, 0};
        int nhas = 0;
        if (cur.cnt == 0) {  /* internal */
          const uint32_t c1 = nodes[cur.ref].first + 1;
          const int spine = nodes[c1].count == 0;
          expand(cur.ref, o, inv, dist, &next, &nhas, stk, &sp);
          if (spine && nhas && next.cnt == 0 && next.ref == c1) {  /* c1 passed: its pair came with this step */
            Ent n2 = {0, 0};
            int h2 = 0;
            expand(c1, o, inv, dist, &n2, &h2, stk, &sp);
            next = n2;
            nhas = h2;
          } else if (!spine && sched >= 1 && sp > 0 && stk[sp - 1].cnt == 0) {  /* the spine slot expands the top */
            const Ent top = stk[--sp];
            Ent n2 = {0, 0};
            int h2 = 0;
            expand(top.ref, o, inv, dist, &n2, &h2, stk, &sp);
            if (h2) {
              if (nhas) stk[sp++] = n2;
              else next = n2, nhas = 1;
            }
          }
        } else {  /* leaf: up to two triangles */
          const uint32_t n = cur.cnt < 2 ? cur.cnt : 2;
          for (uint32_t k = 0; k < n && !hit; ++k) {
            g_tests += 1;
            hit = tri(tris + 9 * (size_t)(cur.ref + k), o, d, dist);
          }
          if (cur.cnt > n) next.ref = cur.ref + n, next.cnt = cur.cnt - n, nhas = 1;
          if (!hit && sched >= 2 && cur.cnt == 1 && sp > 0 && stk[sp - 1].cnt == 0) {
            const Ent top = stk[--sp];
            Ent n2 = {0, 0};
            int h2 = 0;
            expand(top.ref, o, inv, dist, &n2, &h2, stk, &sp);
            if (h2) {
              if (nhas) stk[sp++] = n2;
              else next = n2, nhas = 1;
            }
          }
        }
        if (hit) break;
        if (!nhas && sp > 0) next = stk[--sp], nhas = 1;  /* the pop (a pushed entry still passes) */
        cur = next;
        has = nhas;
      }
      occl += hit;
    }
    printf("schedule %d: rays %u occluded %.4f sub-steps %.3f node pairs %.3f triangle tests %.3f per ray\n", sched,
           hd[2], (double)occl / hd[2], steps / hd[2], g_pairs / hd[2], g_tests / hd[2]);
  }
  {  /* node pairs expanded by depth (schedule 0), cumulative share: what an LDS copy of the top levels would serve */
    double tot = 0, acc = 0;
    for (int d = 0; d < 64; ++d) tot += g_pairs_by_depth[d];
    printf("node pairs by depth of the expanded node, cumulative share:");
    for (int d = 0; d < 24 && tot > 0; ++d) {
      acc += g_pairs_by_depth[d];
      printf(" %d:%.3f", d, acc / tot);
    }
    printf("\n");
  }
  return 0;
}
