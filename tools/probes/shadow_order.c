/* shadow_order.c -- diagnostic: the cost of a shadow ray's any-hit traversal under three child orders.
 *
 * CheckLightOccluded (raytrace_compute.glsl:167-176) only uses CheckHit(...).hit: whether some triangle with
 * 1e-5 < t < |light - p| exists along the ray.  That answer does not depend on the order in which the BVH is
 * walked, so a shadow ray may visit either child first.  This tool counts, per shadow ray, the node pairs
 * expanded and the triangles tested until the first accepted triangle (or the end), for
 *   order 0: the reference's (right child c1 first: ray_intersects.glsl:99-133),
 *   order 1: the nearer child first (larger entry distance pushed),
 *   order 2: the farther child first.
 * Plain fp32 here (it estimates step counts; the kernels' exact arithmetic is not needed for that).
 *
 * Input (binary, little endian): u32 n_nodes, u32 n_tris, u32 n_rays; n_nodes x 32-B std430 BVHNode
 * (min xyz, first, max xyz, count); n_tris x 9 f32 (v0 v1 v2, BVH order); n_rays x 7 f32 (o, d, tmax).
 * Output: one line per order: rays, occluded, mean node pairs, mean triangle tests.
 *   gcc -O2 -o /tmp/shadow_order tools/probes/shadow_order.c -lm && /tmp/shadow_order rays.bin   (tools/probes/shadow_order.py)
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
  for (int order = 0; order < 3; ++order) {
    double pairs = 0, tests = 0;
    long occl = 0;
    for (uint32_t r = 0; r < hd[2]; ++r) {
      const float* o = rays + 7 * (size_t)r;
      const float* d = o + 3;
      const float dist = o[6];
      float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
      uint32_t stk[128];
      int sp = 0, hit = 0;
      if (box(&nodes[0], o, inv) < dist) stk[sp++] = 0;
      while (sp > 0 && !hit) {
        const Node* n = &nodes[stk[--sp]];
        if (n->count > 0) {
          for (uint32_t i = 0; i < n->count && !hit; ++i) {
            tests += 1;
            hit = tri(tris + 9 * (size_t)(n->first + i), o, d, dist);
          }
          continue;
        }
        pairs += 1;
        const uint32_t c0 = n->first, c1 = c0 + 1;
        const float b0 = box(&nodes[c0], o, inv), b1 = box(&nodes[c1], o, inv);
        const int v0 = b0 < dist, v1 = b1 < dist;
        uint32_t first = c1, second = c0;  /* order 0: c1 visited first (pushed last) */
        if (order == 1 && v0 && v1 && b0 < b1) first = c0, second = c1;
        if (order == 2 && v0 && v1 && b0 > b1) first = c0, second = c1;
        const int vf = first == c1 ? v1 : v0, vs = first == c1 ? v0 : v1;
        if (vs && sp < 128) stk[sp++] = second;
        if (vf && sp < 128) stk[sp++] = first;
      }
      occl += hit;
    }
    printf("order %d (%s): rays %u occluded %.4f node pairs %.3f triangle tests %.3f per ray\n", order,
           order == 0 ? "reference, c1 first" : order == 1 ? "nearer first" : "farther first", hd[2],
           (double)occl / hd[2], pairs / hd[2], tests / hd[2]);
  }
  return 0;
}
