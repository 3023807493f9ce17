// shading.hpp -- GetRayColor's shading: spheres, lights, the direct-light and indirect
// BRDFs (shaders/brdf.glsl, raytrace_compute.glsl) in the arithmetic contract.
#pragma once

#include "device_common.hpp"
#include "traversal.hpp"

namespace srt {
using namespace dev;

// Texels are kept as the file's bytes, RGBA8 (SRT_TEX8, round 5: 4 B a texel instead of 16), and a
// channel c is read as c / 255 -- the contract's value, the correctly rounded quotient -- by q = c * RN(1/255)
// and one Markstein correction q + (c - 255 q) / 255 with the residual exact in an FMA: equal to c / 255.0f
// for all 256 values (checked exactly in tests/test_producers.py).
#ifndef SRT_TEX8
#define SRT_TEX8 1
#endif
__device__ __forceinline__ float unorm8(uint32_t p, int sh) {
  constexpr float kInv255 = 0.003921568859368563f;  // RN(1 / 255)
  const float c = (float)((p >> sh) & 255u);
  const float q = c * kInv255;
  return __builtin_fmaf(__builtin_fmaf(-255.0f, q, c), kInv255, q);
}

// texture(sampler2D, vec2(s, t)).xyz at level 0, GL_LINEAR, GL_REPEAT: the
// sampling contract of scene.cpp TextureSample
__device__ __forceinline__ f3 texture_sample(const KParams& kp, uint32_t tex, float s, float t) {
  const uint4 info = kp.tex_info[tex];
  const int w = (int)info.y, h = (int)info.z;
  if (!(__builtin_fabsf(s) <= 3.402823466e38f)) s = 0.0f;
  if (!(__builtin_fabsf(t) <= 3.402823466e38f)) t = 0.0f;
  s = s - __builtin_floorf(s);
  t = t - __builtin_floorf(t);
  const float x = s * (float)w - 0.5f, y = t * (float)h - 0.5f;
  const float fx = __builtin_floorf(x), fy = __builtin_floorf(y);
  const float a = x - fx, b = y - fy;
  int i0 = (int)fx, j0 = (int)fy;
  int i1 = i0 + 1, j1 = j0 + 1;
  i0 = i0 < 0 ? w - 1 : i0;
  j0 = j0 < 0 ? h - 1 : j0;
  i1 = i1 >= w ? 0 : i1;
  j1 = j1 >= h ? 0 : j1;
  const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
#if SRT_TEX8
  const uint32_t* T = kp.tex_texels8 + info.x;
  const uint32_t p00 = T[(uint32_t)j0 * w + i0], p10 = T[(uint32_t)j0 * w + i1];
  const uint32_t p01 = T[(uint32_t)j1 * w + i0], p11 = T[(uint32_t)j1 * w + i1];
  const f3 t00 = mk(unorm8(p00, 0), unorm8(p00, 8), unorm8(p00, 16));
  const f3 t10 = mk(unorm8(p10, 0), unorm8(p10, 8), unorm8(p10, 16));
  const f3 t01 = mk(unorm8(p01, 0), unorm8(p01, 8), unorm8(p01, 16));
  const f3 t11 = mk(unorm8(p11, 0), unorm8(p11, 8), unorm8(p11, 16));
#else
  const float4* T = kp.tex_texels + info.x;
  const float4 t00 = T[(uint32_t)j0 * w + i0], t10 = T[(uint32_t)j0 * w + i1];
  const float4 t01 = T[(uint32_t)j1 * w + i0], t11 = T[(uint32_t)j1 * w + i1];
#endif
  return mk(((w00 * t00.x + w10 * t10.x) + w01 * t01.x) + w11 * t11.x,
            ((w00 * t00.y + w10 * t10.y) + w01 * t01.y) + w11 * t11.y,
            ((w00 * t00.z + w10 * t10.z) + w01 * t01.z) + w11 * t11.z);
}

// TriangleToSupportedMat's texture branch (raytrace_utils.glsl:144-166) for
// hit triangle `ht` (records A, B, C: v0, e1 = v1 - v0, e2 = v2 - v0) at
// distance `dist` along the world ray: model_p in the frame of the BVH that
// owns the triangle (raytrace_compute.glsl:155), barycentrics, uv, sample.
__device__ __forceinline__ f3 mesh_texture_albedo(const KParams& kp, uint32_t tex, uint32_t ht, float4 A, float4 B,
                                               float4 C, float dist, f3 ro, f3 rd) {
  if (tex >= kp.n_tex) return mk(0.0f, 0.0f, 0.0f);  // unknown handle
  uint32_t hb = 0;
  for (uint32_t j = 0; j < kp.bvh_count; ++j) {  // pad0/pad1: the record's triangle range
    const srt_bvh_record& r = kp.bvhs[j];
    if (ht - r.pad0 < r.pad1 - r.pad0) hb = j;
  }
  const srt_bvh_record& b = kp.bvhs[hb];
  const f3 to = xform(b.frame, ro, 1.0f), td = xform(b.frame, rd, 0.0f);
  const f3 mp = (dist * td) + to;
  const f3 v0 = mk(A.x, A.y, A.z), v0v1 = mk(A.w, B.x, B.y), v0v2 = mk(B.z, B.w, C.x);
  const f3 v0p = mp - v0;
  const float d00 = dot(v0v1, v0v1), d01 = dot(v0v1, v0v2), d11 = dot(v0v2, v0v2);
  const float d20 = dot(v0p, v0v1), d21 = dot(v0p, v0v2);
  const float denom = 1.0f / (d00 * d11 - d01 * d01);
  const float v = (d11 * d20 - d01 * d21) * denom;
  const float w = (d00 * d21 - d01 * d20) * denom;
  const float u = 1.0f - v - w;
  const float4 uv01 = kp.tri_uv[2 * ht], uv2 = kp.tri_uv[2 * ht + 1];
  const float s = (u * uv01.x + v * uv01.z) + w * uv2.x;
  const float t = (u * uv01.y + v * uv01.w) + w * uv2.y;
  return texture_sample(kp, tex, s, t);
}

// raytrace_compute.glsl:93-120 SphereHit
__device__ __forceinline__ bool sphere_hit(f3 ro, f3 rd, f3 pos, float radius, float mn, float mx, float& t) {
  const f3 oc = pos - ro;
  const float ld = length(rd);
  const float a = ld * ld;
  const float h = dot(rd, oc);
  const float loc = length(oc);
  const float cc = loc * loc - (radius * radius);
  const float disc = h * h - a * cc;
  if (disc < 0.0f) return false;
  const float sq = __builtin_sqrtf(disc);
  float root = div_rn(h - sq, a);
  if (!(mn < root && root < mx)) {
    root = div_rn(h + sq, a);
    if (!(mn < root && root < mx)) return false;
  }
  t = root;
  return true;
}

// CheckHit over the five spheres (raytrace_compute.glsl:132-141): index of the
// closest sphere (dist updated) or, with `any`, of the first sphere hit; -1 if none.
__device__ __forceinline__ int trace_spheres(f3 ro, f3 rd, float mn, float& dist, bool any) {
  int best = -1;
  for (int i = 0; i < 5; ++i) {
    f3 pos; float radius; Mat m;
    sphere_data(i, pos, radius, m);
    float t;
    if (sphere_hit(ro, rd, pos, radius, mn, dist, t)) {
      best = i;
      dist = t;
      if (any) break;
    }
  }
  return best;
}

template <bool COUNT>
__device__ __forceinline__ LightRec load_light(const KParams& kp, Counters& c, int idx) {
  bump<COUNT>(c, ST_LIGHTS);
  const int i = (idx >= 0 && idx < kp.light_records) ? idx : kp.light_records;  // zero record
  float4 a, b;
  if (kp.lights_lds) {
    a = lds4((uint32_t)(kp.lights_base_f4 + 2 * i) << 4);
    b = lds4((uint32_t)(kp.lights_base_f4 + 2 * i + 1) << 4);
  } else {
    a = kp.lights[2 * i];
    b = kp.lights[2 * i + 1];
  }
  return LightRec{mk(a.x, a.y, a.z), a.w, mk(b.x, b.y, b.z)};
}

__device__ __forceinline__ float ggxD(float NdotH, float rough) {
  const float a2 = rough * rough;
  const float d = ((NdotH * a2 - NdotH) * NdotH + 1.0f);
  return div_rn(a2, fmx(0.001f, (d * d * 3.1415926535897f)));
}
__device__ __forceinline__ float ggxDNew(float NdotH, float alphaSquared) {
  const float b = ((alphaSquared - 1.0f) * NdotH * NdotH + 1.0f);
  return div_rn(alphaSquared, fmx(0.001f, (3.1415926535897f * b * b)));
}
__device__ __forceinline__ float ggxSchlickMasking(float NdotL, float NdotV, float rough) {
  const float k = rough * rough / 2.0f;
  const float gv = div_rn(NdotV, fmx(0.001f, (NdotV * (1.0f - k) + k)));
  const float gl = div_rn(NdotL, fmx(0.001f, (NdotL * (1.0f - k) + k)));
  return __builtin_fabsf(gv * gl);
}
__device__ __forceinline__ float smithGAlpha(float alpha, float NdotS) {
  return div_rn(NdotS, fmx(0.0001f, alpha) * __builtin_sqrtf(1.0f - fmn(0.99999f, NdotS * NdotS)));
}
__device__ __forceinline__ float smithLambda(float a) {
  return (-1.0f + __builtin_sqrtf(1.0f + recip_exact(fmx(0.001f, a * a)))) * 0.5f;
}
__device__ __forceinline__ float smithG2(float alpha, float NdotL, float NdotV) {
  const float aL = smithGAlpha(alpha, NdotL);
  const float aV = smithGAlpha(alpha, NdotV);
  return recip_exact(1.0f + smithLambda(aL) + smithLambda(aV));
}

// brdf.glsl:200-224 SampleDirect up to the shadow factor: returns
// (ggxTerm + NdotL * albedo / pi) and the light term's unshadowed factors.
// Ld = getLightData's direction, H = its guarded half vector with V (computed
// by the caller, shared with the shadow ray; li = intensity * falloff there too)
__device__ f3 sample_direct_brdf(const Hit& hit, f3 Vv, f3 Ld, f3 H) {
  const f3 N = hit.normal;
  const float NdotL = sat(dot(N, Ld));
  const float NdotH = sat(dot(N, H));
  const float LdotH = sat(dot(Ld, H));
  const float NdotV = sat(dot(N, Vv));
  const float rough = hit.mat.roughness;
  const float D = ggxD(NdotH, rough);
  const float G = ggxSchlickMasking(NdotL, NdotV, rough);
  const f3 F = schlickFresnel(hit.mat.specular, LdotH);
  const f3 ggx = (F * (D * G)) / (4.0f * fmx(0.001f, NdotV));
  const f3 diff = (NdotL * hit.mat.albedo) / 3.1415926535897f;
  return ggx + diff;
}

// brdf.glsl:226-237 SampleDirectNew (GetAllBRDFValues :173-198, EvalSpecular :139-145
// with ggxNormalDistributionNew's arguments swapped as in the reference, EvalDiffuse :134-137)
// H = normalize(L + Vv) (computed by the caller as normalize(Vv + L))
__device__ f3 sample_direct_new(const Hit& hit, f3 Vv, f3 L, f3 H) {
  const f3 N = hit.normal;
  const float NdotL = sat(dot(N, L));
  const float NdotV = sat(dot(N, Vv));
  const float LdotH = sat(dot(L, H));
  const float NdotH = sat(dot(N, H));
  const f3 specF0 = specularF0(hit.mat.albedo, hit.mat.metalness);
  const f3 diffRefl = hit.mat.albedo * (1.0f - hit.mat.metalness);
  const float alpha = hit.mat.roughness * hit.mat.roughness;
  const float alphaSq = alpha * alpha;
  const f3 F = fresnelSchlickNew(specF0, shadowedF90(specF0), LdotH);
  const float D = ggxDNew(fmx(0.00001f, alphaSq), NdotH);
  const float G = smithG2(alpha, NdotL, NdotV);
  const float denom = 4.0f * fmx(NdotL, 0.001f) * fmx(NdotV, 0.001f);
  const f3 spec = (((F * G) * D) / fmx(denom, 0.001f)) * NdotL;
  const float oneOverPi = 1.0f / 3.1415926535897f;
  const f3 diff = diffRefl * (oneOverPi * NdotL);
  return ((mk(1.0f, 1.0f, 1.0f) - F) * diff) + spec;
}

// brdf.glsl:279-288
__device__ float brdf_probability(const Mat& m, f3 Vv, f3 N) {
  const float sF0 = luminance(specularF0(m.albedo, m.metalness));
  const float dR = luminance(m.albedo * (1.0f - m.metalness));
  const f3 f0 = mk(sF0, sF0, sF0);
  const float F = sat(luminance(fresnelSchlickNew(f0, shadowedF90(f0), fmx(0.0f, dot(Vv, N)))));
  const float diffuse = dR * (1.0f - F);
  const float p = div_rn(F, fmx(0.0001f, (F + diffuse)));
  return clampf(p, 0.1f, 0.9f);
}

// brdf.glsl:81-99 SampleSpecularHalfVec given its two uniform draws
__device__ __forceinline__ f3 specular_half(float rx, float ry, float rough, f3 N) {
  const f3 B = perpendicular(N);
  const f3 T = cross(B, N);
  const float a2 = rough * rough;
  const float cosT = __builtin_sqrtf(fmx(0.0f, div_rn(1.0f - rx, (a2 - 1.0f) * rx + 1.0f)));
  const float sinT = __builtin_sqrtf(fmx(0.0f, 1.0f - cosT * cosT));
  const float phi = ry * 3.1415926535897f * 2.0f;
  return ((T * (sinT * cos_f(phi))) + (B * (sinT * sin_f(phi)))) + (N * cosT);
}

__device__ __forceinline__ f3 reflect3(f3 I, f3 N) { return I - N * (2.0f * dot(N, I)); }

#define DIFFUSE_BRDF 1
#define SPECULAR_BRDF 2

// brdf.glsl:239-277 SampleIndirectNew with its uniform draws r1 = U(p.xy),
// r2 = U(p.yz) supplied (SampleDiffuse :60-74 and SampleSpecularHalfVec :81-99
// both draw exactly these two numbers).
// SampleIndirectNew (brdf.glsl:239-277).  The diffuse branch (SampleDiffuse +
// its Fresnel weight from SampleSpecularHalfVec) and the specular branch
// (SampleSpecularMicrofacet) share their basis, phi = 2*pi*r2 with its cos/sin
// ((2*pi)*r2 and (r2*pi)*2 round identically: the factor 2 is exact), the GGX
// half vector of (r1, r2) and one Fresnel evaluation, so lanes of a wave that
// took different branches compute those once; every value is the reference's.
__device__ bool sample_indirect(const Hit& hit, f3 Vv, int type, float r1, float r2, f3& dir, f3& weight) {
  const f3 N = hit.normal;
  if (dot(N, Vv) <= 0.0f) return false;
  const f3 specF0 = specularF0(hit.mat.albedo, hit.mat.metalness);
  const f3 B = perpendicular(N);
  const f3 T = cross(B, N);
  const float phi = 2.0f * 3.1415926535897f * r2;
  const float cphi = cos_f(phi), sphi = sin_f(phi);
  // SampleSpecularHalfVec(r1, r2, roughness, N) (brdf.glsl:81-99)
  const float a2 = hit.mat.roughness * hit.mat.roughness;
  const float cosT = __builtin_sqrtf(fmx(0.0f, div_rn(1.0f - r1, (a2 - 1.0f) * r1 + 1.0f)));
  const float sinT = __builtin_sqrtf(fmx(0.0f, 1.0f - cosT * cosT));
  const f3 Hs = ((T * (sinT * cphi)) + (B * (sinT * sphi))) + (N * cosT);
  f3 nd, w0;
  float fx;
  if (type == DIFFUSE_BRDF) {
    // SampleDiffuse (brdf.glsl:60-74)
    const float r = __builtin_sqrtf(__builtin_fabsf(r1));
    nd = ((T * (r * cphi)) + (B * (r * sphi))) + (N * __builtin_sqrtf(__builtin_fabsf(1.0f - r1)));
    w0 = hit.mat.albedo * (1.0f - hit.mat.metalness);
    fx = fmx(0.00001f, fmn(1.0f, dot(Vv, Hs)));  // VdotH
  } else {
    // brdf.glsl:102-132 SampleSpecularMicrofacet
    const float alpha = hit.mat.roughness * hit.mat.roughness;
    const float alphaSq = alpha * alpha;
    f3 H = Hs;
    if (alpha == 0.0f) {
      const f3 Lt = reflect3(-Vv, N);
      H = normalize(-Vv + Lt);
    }
    const f3 L = reflect3(-Vv, H);
    fx = fmx(0.00001f, fmn(1.0f, dot(H, L)));  // HdotL
    const float NdotL = fmx(0.00001f, fmn(1.0f, dot(N, L)));
    const float N2 = NdotL * NdotL;
    w0 = mk(div_rn(2.0f, __builtin_sqrtf(div_rn((alphaSq * (1.0f - N2)) + N2, N2)) + 1.0f), 0.0f, 0.0f);
    nd = L;
  }
  const f3 F = fresnelSchlickNew(specF0, shadowedF90(specF0), fx);
  if (type == DIFFUSE_BRDF) weight = w0 * (mk(1.0f, 1.0f, 1.0f) - F);
  else weight = F * w0.x;
  if (luminance(weight) == 0.0f) return false;
  dir = normalize(nd);
  if (dot(N, dir) <= 0.0f) return false;
  return true;
}

}  // namespace srt
