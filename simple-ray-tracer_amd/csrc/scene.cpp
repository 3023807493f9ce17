// scene.cpp -- scene producers: OBJ/MTL reader, midpoint-split BVH, flattening.
//
// Clean-room restatement of the reference's input producers, reproducing
// their output arrays bit for bit (SURVEY.md 8a "Host-side inputs"):
//   src/asset_utils/model_loader.cpp:20-365   (LoadObject / ParseOBJ / ParseMTL /
//                                               ConvertCPUGeometryToModel)
//   include/intersection_utils/bvh.h:40-148    (BVH ctor, UpdateNodeBounds, Subdivide)
//   src/asset_utils/gpu_loader.cpp:63-133      (UploadModelDataToGPU flattening)
// All float arithmetic is plain IEEE fp32 in source order (the reference is
// built by g++ for x86-64 without -march, so SSE and no FMA contraction).
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <thread>
#include <unordered_map>
#include <zlib.h>

#include "srt_internal.hpp"

namespace srt {

namespace {

const char* kWs = " \n\r\t";

void Trim(std::string* line) {
  line->erase(0, line->find_first_not_of(kWs));
  const auto last = line->find_last_not_of(kWs);
  line->erase(last == std::string::npos ? 0 : last + 1);
}

struct Face {
  uint32_t v[3];
  uint32_t t[3] = {0, 0, 0};  // vt indices, valid when t_ok (IsTextureIdxsValid)
  bool t_ok = false;
};

struct SubGeometry {
  std::string material;
  std::vector<Face> faces;
};

// model_loader.cpp:35-177 ParseOBJ
bool ParseOBJ(const std::string& path, std::vector<Vec3>* vertices, std::vector<std::pair<float, float>>* uvs,
              std::vector<SubGeometry>* geos, std::vector<std::string>* mtl_files, uint64_t* dropped,
              std::string* err) {
  auto index = [&](const std::string& tok, uint32_t* out) {
    char* end = nullptr;
    const long idx = std::strtol(tok.c_str(), &end, 10);
    if (end == tok.c_str()) {
      *err = "bad face index '" + tok + "' in " + path;
      return false;  // std::stol throws in the reference
    }
    *out = static_cast<uint32_t>(idx - 1);  // OBJ indices are 1-based
    return true;
  };
  std::ifstream file(path);
  if (!file) {
    *err = "cannot open " + path;
    return false;
  }
  SubGeometry cur;
  std::string line;
  while (std::getline(file, line)) {
    Trim(&line);
    if (line.empty() || line[0] == '#') continue;
    std::istringstream ls(line);
    std::string prefix;
    ls >> prefix;
    if (prefix == "v") {
      Vec3 v;
      if (ls >> v.x >> v.y >> v.z) vertices->push_back(v);  // libstdc++ num_get, as the reference
    } else if (prefix == "vt") {  // model_loader.cpp:65-71
      float a, b;
      if (ls >> a >> b) uvs->emplace_back(a, b);
    } else if (prefix == "f") {  // model_loader.cpp:82-143: v/vt/vn per corner
      std::vector<uint32_t> vi, ti;
      std::string tok;
      while (ls >> tok) {
        const auto s1 = tok.find('/');
        const std::string v = tok.substr(0, s1);
        std::string vt;
        if (s1 != std::string::npos) {
          const auto s2 = tok.find('/', s1 + 1);
          vt = tok.substr(s1 + 1, s2 == std::string::npos ? std::string::npos : s2 - s1 - 1);
        }
        uint32_t idx;
        if (!v.empty()) {
          if (!index(v, &idx)) return false;
          vi.push_back(idx);
        }
        if (!vt.empty()) {
          if (!index(vt, &idx)) return false;
          ti.push_back(idx);
        }
      }
      if (vi.size() != 3 && vi.size() != 4) {
        ++*dropped;  // "Unexpected face vertex count" (model_loader.cpp:110-113)
        continue;
      }
      Face f1{{vi[0], vi[1], vi[2]}};
      if (ti.size() > 2) {
        f1.t[0] = ti[0]; f1.t[1] = ti[1]; f1.t[2] = ti[2];
        f1.t_ok = true;
      }
      cur.faces.push_back(f1);
      if (vi.size() == 4) {
        Face f2{{vi[0], vi[2], vi[3]}};
        if (ti.size() == 4) {
          f2.t[0] = ti[0]; f2.t[1] = ti[2]; f2.t[2] = ti[3];
          f2.t_ok = true;
        }
        cur.faces.push_back(f2);
      }
    } else if (prefix == "usemtl") {
      if (!cur.material.empty()) {
        geos->push_back(std::move(cur));
        cur = SubGeometry();
      }
      std::string name;
      ls >> name;
      cur.material = name;
    } else if (prefix == "mtllib") {
      std::string name;
      ls >> name;
      mtl_files->push_back(name);
    }
    // vn never reaches the GPU; s / o / g and unknown prefixes are ignored.
  }
  if (!cur.material.empty()) geos->push_back(std::move(cur));
  else *dropped += cur.faces.size();  // trailing faces without a material are dropped
  return true;
}

// model_loader.cpp:179-278 ParseMTL.  Materials keep first-definition order
// (the reference's unordered_map order is renderer-invisible).
void ParseMTL(const std::string& folder, const std::string& file_name, std::vector<std::string>* names,
              std::vector<Material>* mats) {
  std::ifstream file(folder + file_name);
  if (!file) return;  // "Cannot open file" and continue
  long current = -1;
  std::string line;
  while (std::getline(file, line)) {
    Trim(&line);
    if (line.empty() || line[0] == '#') continue;
    std::istringstream ls(line);
    std::string prefix;
    ls >> prefix;
    if (prefix == "newmtl") {
      std::string name;
      ls >> name;
      bool dup = false;
      for (const auto& n : *names) dup |= (n == name);
      if (!dup) {  // a duplicate name leaves `current` on the previous material
        names->push_back(name);
        mats->emplace_back();
        current = static_cast<long>(mats->size()) - 1;
      }
      continue;
    }
    if (current < 0) continue;
    Material& m = (*mats)[current];
    if (prefix == "map_Kd") {
      std::string tex;
      ls >> tex;
      m.use_texture = true;
      m.texture_path = folder + "/" + tex;
    } else if (prefix == "Kd") {
      Vec3 d;
      ls >> d.x >> d.y >> d.z;  // the reference's glm::vec3 is indeterminate where nothing is read: 0 here
      m.diffuse = d;
    } else if (prefix == "Ks") {
      Vec3 s;
      ls >> s.x >> s.y >> s.z;
      m.specular = s;
    } else if (prefix == "Ns") {
      float e = 0.f;
      ls >> e;
      m.specular_ex = e;
    }
  }
}

// ---------------------------------------------------------------------------
// BVH (bvh.h:40-148) over triangles, with model_loader.cpp:333-352 centre/bounds
// ---------------------------------------------------------------------------
// Runs body(i) for i in [0, n) on `threads` threads (dynamic, one index at a time).
template <class F>
void ParallelFor(size_t n, int threads, F body) {
  if (threads <= 1 || n <= 1) {
    for (size_t i = 0; i < n; ++i) body(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> pool;
  const int t = (int)std::min<size_t>((size_t)threads, n);
  for (int k = 0; k < t; ++k)
    pool.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) body(i);
    });
  for (auto& th : pool) th.join();
}

// bvh.h:40-148.  The reference builds recursively: a node that splits gets its
// child pair at the next free index (pre-order), then its left subtree is
// built completely, then its right.  So every subtree's pairs occupy one
// contiguous block of indices, and the tree can be built in parallel with the
// same bits: the top levels are split level by level (nodes of a level in
// parallel: their primitive ranges are disjoint), the subtrees below are built
// in parallel with local pre-order numbering, and one pre-order walk then gives
// every block its global offset.  BuildBVH uses it above kParallelMinPrims
// primitives (SRT_BVH_THREADS, default min(16, hardware threads); 1 = serial).
class BvhBuilder {
 public:
  BvhBuilder(Model* m, int threads) : m_(m), threads_(threads) {}

  void Build() {
    const size_t n = m_->prims.size();
    idx_.resize(n);
    centers_.resize(n);
    bmin_.resize(n);
    bmax_.resize(n);
    const size_t chunk = 1 << 16;
    ParallelFor((n + chunk - 1) / chunk, threads_, [&](size_t c) {
      for (size_t i = c * chunk; i < std::min(n, (c + 1) * chunk); ++i) {
        idx_[i] = static_cast<uint32_t>(i);
        const Triangle& t = m_->prims[i];
        const Vec3 p0 = Pos(t.vertex_idxs[0]), p1 = Pos(t.vertex_idxs[1]), p2 = Pos(t.vertex_idxs[2]);
        // (p0 + p1 + p2) / 3.0f
        centers_[i] = Vec3((p0.x + p1.x + p2.x) / 3.0f, (p0.y + p1.y + p2.y) / 3.0f, (p0.z + p1.z + p2.z) / 3.0f);
        bmin_[i] = vmin(vmin(p0, p1), p2);
        bmax_[i] = vmax(vmax(p0, p1), p2);
      }
    });
    BVHNode root;
    root.first_child = 0;
    root.first_prim_index = 0;
    root.prim_count = static_cast<uint32_t>(n);
    UpdateBounds(&root);
    uint32_t max_depth = 0, leaves = 0;
    std::vector<BVHNode> nodes;
    if (threads_ <= 1 || n < kParallelMinPrims) {
      BuildSubtree(root, &nodes, &max_depth, &leaves);
    } else {
      BuildParallel(root, &nodes, &max_depth, &leaves);
    }
    std::vector<Triangle> np(n);
    ParallelFor((n + chunk - 1) / chunk, threads_, [&](size_t c) {
      for (size_t i = c * chunk; i < std::min(n, (c + 1) * chunk); ++i) np[i] = m_->prims[idx_[i]];
    });
    m_->prims = std::move(np);
    m_->prim_input = idx_;
    m_->nodes = std::move(nodes);
    m_->max_depth = max_depth;
    m_->leaves = leaves;
  }

  static constexpr size_t kParallelMinPrims = 65536;

 private:
  Vec3 Pos(uint32_t v) const {
    const srt_vertex& sv = m_->vertices[v];
    return Vec3(sv.vertex[0], sv.vertex[1], sv.vertex[2]);
  }

  // bvh.h:80-96
  void UpdateBounds(BVHNode* node) const {
    node->min_bounds = Vec3(std::numeric_limits<float>::max(), std::numeric_limits<float>::max(),
                            std::numeric_limits<float>::max());
    node->max_bounds = Vec3(std::numeric_limits<float>::lowest(), std::numeric_limits<float>::lowest(),
                            std::numeric_limits<float>::lowest());
    for (uint32_t i = 0; i < node->prim_count; ++i) {
      const uint32_t p = idx_[node->first_prim_index + i];
      node->min_bounds = vmin(node->min_bounds, bmin_[p]);
      node->max_bounds = vmax(node->max_bounds, bmax_[p]);
    }
  }

  // bvh.h:98-148: partitions the node's range of idx_ and fills its children
  // (first_child is left to the caller); false when the node stays a leaf
  bool Split(BVHNode* node, BVHNode* left, BVHNode* right) {
    if (node->prim_count <= 2) return false;
    const Vec3 extent(node->max_bounds.x - node->min_bounds.x, node->max_bounds.y - node->min_bounds.y,
                      node->max_bounds.z - node->min_bounds.z);
    int axis = 0;
    if (extent.y > extent.x) axis = 1;
    if (extent.z > extent[axis]) axis = 2;
    const float split = node->min_bounds[axis] + extent[axis] * 0.5f;
    uint32_t i = node->first_prim_index;
    uint32_t j = i + node->prim_count - 1;
    while (i <= j && j != static_cast<uint32_t>(-1)) {
      if (centers_[idx_[i]][axis] < split) {
        i++;
      } else {
        std::swap(idx_[i], idx_[j]);
        j--;
      }
    }
    const uint32_t left_count = i - node->first_prim_index;
    if (left_count == 0 || left_count == node->prim_count) return false;
    *left = BVHNode();
    *right = BVHNode();
    left->first_prim_index = node->first_prim_index;
    left->prim_count = left_count;
    right->first_prim_index = i;
    right->prim_count = node->prim_count - left_count;
    node->prim_count = 0;
    UpdateBounds(left);
    UpdateBounds(right);
    return true;
  }

  // The subtree of `root` in the reference's order, numbered locally: out[0] =
  // root, child pairs from 1 on in pre-order.  Depth and leaves are relative.
  void BuildSubtree(const BVHNode& root, std::vector<BVHNode>* out, uint32_t* max_depth, uint32_t* leaves) {
    out->assign(1, root);
    struct Item { uint32_t node; uint32_t depth; };
    std::vector<Item> stack{{0, 0}};
    uint32_t md = 0, lv = 0;
    while (!stack.empty()) {
      const Item it = stack.back();
      stack.pop_back();
      if (it.depth > md) md = it.depth;
      BVHNode l, r;
      BVHNode node = (*out)[it.node];
      if (Split(&node, &l, &r)) {
        const uint32_t li = static_cast<uint32_t>(out->size());
        node.first_child = li;
        (*out)[it.node] = node;
        out->push_back(l);
        out->push_back(r);
        stack.push_back({li + 1, it.depth + 1});
        stack.push_back({li, it.depth + 1});
      } else {
        (*out)[it.node] = node;
        ++lv;
      }
    }
    *max_depth = md;
    *leaves = lv;
  }

  struct TopNode {
    BVHNode node;
    int left = -1;      // index of the left child in top_ (right = left + 1)
    int task = -1;      // subtree built by BuildSubtree
    uint32_t depth = 0;
  };

  void BuildParallel(const BVHNode& root, std::vector<BVHNode>* out, uint32_t* max_depth, uint32_t* leaves) {
    // 1. top levels, level by level, until there is enough independent work
    top_.assign(1, TopNode{root, -1, -1, 0});
    std::vector<int> level{0};
    const size_t want = (size_t)threads_ * 8;
    const uint32_t small = std::max<uint32_t>(4096, (uint32_t)(m_->prims.size() / (want * 4)));
    while (!level.empty() && level.size() < want) {
      std::vector<char> split(level.size(), 0);
      std::vector<BVHNode> kids(2 * level.size());
      ParallelFor(level.size(), threads_, [&](size_t k) {
        TopNode& t = top_[level[k]];
        if (t.node.prim_count <= small) return;  // left for the subtree stage
        split[k] = Split(&t.node, &kids[2 * k], &kids[2 * k + 1]) ? 1 : 2;
      });
      std::vector<int> next;
      for (size_t k = 0; k < level.size(); ++k) {
        if (split[k] != 1) continue;  // 0: a subtree task, 2: a leaf
        const int li = static_cast<int>(top_.size());
        top_[level[k]].left = li;
        const uint32_t d = top_[level[k]].depth + 1;
        top_.push_back(TopNode{kids[2 * k], -1, -1, d});
        top_.push_back(TopNode{kids[2 * k + 1], -1, -1, d});
        next.push_back(li);
        next.push_back(li + 1);
      }
      for (size_t k = 0; k < level.size(); ++k)
        if (split[k] == 0) tasks_.push_back(level[k]);
      level.swap(next);
    }
    for (int t : level) tasks_.push_back(t);
    // 2. the subtrees, largest first
    std::vector<int> order(tasks_.size());
    for (size_t k = 0; k < order.size(); ++k) order[k] = (int)k;
    std::sort(order.begin(), order.end(), [&](int a, int b) {
      return top_[tasks_[a]].node.prim_count > top_[tasks_[b]].node.prim_count;
    });
    sub_.resize(tasks_.size());
    sub_depth_.resize(tasks_.size());
    sub_leaves_.resize(tasks_.size());
    for (size_t k = 0; k < tasks_.size(); ++k) top_[tasks_[k]].task = (int)k;
    ParallelFor(order.size(), threads_, [&](size_t q) {
      const int k = order[q];
      BuildSubtree(top_[tasks_[k]].node, &sub_[k], &sub_depth_[k], &sub_leaves_[k]);
    });
    // 3. global pre-order numbering
    size_t total = 1;
    for (const TopNode& t : top_)
      if (t.left >= 0) total += 2;
    for (const auto& v : sub_) total += v.size() - 1;
    out->assign(total, BVHNode());
    next_ = 1;
    *max_depth = 0;
    *leaves = 0;
    Emit(0, 0, out, max_depth, leaves);
  }

  void Emit(int ti, uint32_t g, std::vector<BVHNode>* out, uint32_t* max_depth, uint32_t* leaves) {
    const TopNode& t = top_[ti];
    if (t.task >= 0) {
      const std::vector<BVHNode>& loc = sub_[t.task];
      const uint32_t base = next_;  // local index k >= 1 -> base + k - 1
      next_ += static_cast<uint32_t>(loc.size() - 1);
      auto remap = [&](BVHNode n) {
        if (n.prim_count == 0) n.first_child = base + n.first_child - 1;
        return n;
      };
      (*out)[g] = remap(loc[0]);
      for (size_t k = 1; k < loc.size(); ++k) (*out)[base + k - 1] = remap(loc[k]);
      *max_depth = std::max(*max_depth, t.depth + sub_depth_[t.task]);
      *leaves += sub_leaves_[t.task];
    } else if (t.left >= 0) {
      const uint32_t pair = next_;
      next_ += 2;
      BVHNode n = t.node;
      n.first_child = pair;
      (*out)[g] = n;
      *max_depth = std::max(*max_depth, t.depth);
      Emit(t.left, pair, out, max_depth, leaves);
      Emit(t.left + 1, pair + 1, out, max_depth, leaves);
    } else {
      (*out)[g] = t.node;
      *max_depth = std::max(*max_depth, t.depth);
      ++*leaves;
    }
  }

  Model* m_;
  int threads_;
  std::vector<uint32_t> idx_;
  std::vector<Vec3> centers_, bmin_, bmax_;
  std::vector<TopNode> top_;
  std::vector<int> tasks_;
  std::vector<std::vector<BVHNode>> sub_;
  std::vector<uint32_t> sub_depth_, sub_leaves_;
  uint32_t next_ = 0;
};

// ---------------------------------------------------------------------------
// Minimal PNG reader (8-bit, non-interlaced) for map_Kd textures.
// ---------------------------------------------------------------------------
uint32_t Be32(const unsigned char* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}

bool DecodePng(const std::string& path, int* w, int* h, int* ch, std::vector<unsigned char>* px,
               std::string* err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) { *err = "cannot open texture " + path; return false; }
  std::vector<unsigned char> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (d.size() < 8 || std::memcmp(d.data(), sig, 8) != 0) { *err = "not a PNG: " + path; return false; }
  size_t pos = 8;
  int bitdepth = 0, ctype = 0, interlace = 0;
  std::vector<unsigned char> idat, plte, trns;
  while (pos + 12 <= d.size()) {
    const uint32_t len = Be32(&d[pos]);
    const std::string type(reinterpret_cast<const char*>(&d[pos + 4]), 4);
    if (pos + 12 + len > d.size()) break;
    const unsigned char* body = &d[pos + 8];
    if (type == "IHDR") {
      *w = static_cast<int>(Be32(body));
      *h = static_cast<int>(Be32(body + 4));
      bitdepth = body[8];
      ctype = body[9];
      interlace = body[12];
    } else if (type == "PLTE") {
      plte.assign(body, body + len);
    } else if (type == "tRNS") {
      trns.assign(body, body + len);
    } else if (type == "IDAT") {
      idat.insert(idat.end(), body, body + len);
    } else if (type == "IEND") {
      break;
    }
    pos += 12 + len;
  }
  if (bitdepth != 8 || interlace != 0) { *err = "unsupported PNG (bit depth/interlace): " + path; return false; }
  int in_ch = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
  if (in_ch == 0) { *err = "unsupported PNG colour type: " + path; return false; }
  const size_t stride = size_t(*w) * in_ch;
  std::vector<unsigned char> raw((stride + 1) * size_t(*h));
  uLongf rawlen = raw.size();
  if (uncompress(raw.data(), &rawlen, idat.data(), idat.size()) != Z_OK || rawlen != raw.size()) {
    *err = "PNG inflate failed: " + path;
    return false;
  }
  std::vector<unsigned char> img(stride * size_t(*h));
  for (int y = 0; y < *h; ++y) {
    const unsigned char ft = raw[y * (stride + 1)];
    const unsigned char* src = &raw[y * (stride + 1) + 1];
    unsigned char* dst = &img[y * stride];
    const unsigned char* up = y > 0 ? &img[(y - 1) * stride] : nullptr;
    for (size_t x = 0; x < stride; ++x) {
      const int a = x >= size_t(in_ch) ? dst[x - in_ch] : 0;
      const int b = up ? up[x] : 0;
      const int c = (up && x >= size_t(in_ch)) ? up[x - in_ch] : 0;
      int v = src[x];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) / 2; break;
        case 4: {
          const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
          v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
          break;
        }
        default: *err = "bad PNG filter: " + path; return false;
      }
      dst[x] = static_cast<unsigned char>(v & 0xFF);
    }
  }
  if (ctype == 3) {  // palette -> RGB(A), as stb_image expands it
    const int out_ch = trns.empty() ? 3 : 4;
    px->resize(size_t(*w) * (*h) * out_ch);
    for (size_t i = 0; i < size_t(*w) * (*h); ++i) {
      const unsigned k = img[i];
      for (int c = 0; c < 3; ++c) (*px)[i * out_ch + c] = (3 * k + c < plte.size()) ? plte[3 * k + c] : 0;
      if (out_ch == 4) (*px)[i * out_ch + 3] = k < trns.size() ? trns[k] : 255;
    }
    *ch = out_ch;
  } else {
    *px = std::move(img);
    *ch = in_ch;
  }
  return true;
}

}  // namespace

bool DecodePngTexture(const std::string& path, Texture* out, std::string* err) {
  out->path = path;
  return DecodePng(path, &out->width, &out->height, &out->channels, &out->texels, err);
}

// texture(sampler2D, vec2(s, t)) at level 0 with GL_LINEAR + GL_REPEAT
// (gpu_texture.h:52-58; a compute shader has no derivatives, so lod = 0 and
// the magnification filter applies).  The contract, shared with the kernel
// (shading.hpp texture_sample) and the oracle: fp32 in source order, a
// non-finite coordinate reads as 0, REPEAT as s - floor(s), texel centres at
// (i + 0.5) / size, texels c / 255, and the four weighted texels summed
// (00 + 10) + 01 + 11.  GL_RED samples as (r, 0, 0).  A 2-channel file has no
// defined result in the reference: it uploads the 2-byte texels as GL_RGB
// (gpu_texture.h:39-52), so GL reads byte triples past the image; here it
// samples as (r, g, 0).
void TextureSample(const uint8_t* texels, int width, int height, int channels, float s, float t, float rgb[3]) {
  if (!(std::fabs(s) <= 3.402823466e38f)) s = 0.0f;
  if (!(std::fabs(t) <= 3.402823466e38f)) t = 0.0f;
  s = s - std::floor(s);
  t = t - std::floor(t);
  const float x = s * (float)width - 0.5f, y = t * (float)height - 0.5f;
  const float fx = std::floor(x), fy = std::floor(y);
  const float a = x - fx, b = y - fy;
  int i0 = (int)fx, j0 = (int)fy;
  int i1 = i0 + 1, j1 = j0 + 1;
  i0 = i0 < 0 ? width - 1 : i0;
  j0 = j0 < 0 ? height - 1 : j0;
  i1 = i1 >= width ? 0 : i1;
  j1 = j1 >= height ? 0 : j1;
  const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
  auto texel = [&](int i, int j, int k) -> float {
    if (k >= channels || (k == 2 && channels == 2)) return 0.0f;
    return (float)texels[((size_t)j * width + i) * channels + k] / 255.0f;
  };
  for (int k = 0; k < 3; ++k)
    rgb[k] = ((w00 * texel(i0, j0, k) + w10 * texel(i1, j0, k)) + w01 * texel(i0, j1, k)) + w11 * texel(i1, j1, k);
}

int BvhThreads() {
  if (const char* e = std::getenv("SRT_BVH_THREADS")) return std::max(1, std::atoi(e));
  return (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

void BuildBVH(Model* m) { BvhBuilder(m, BvhThreads()).Build(); }

// model_loader.cpp:20-32 + 280-365
std::unique_ptr<Model> LoadObjectFile(const std::string& obj_path, bool texcoords, std::string* err) {
  std::vector<Vec3> vertices;
  std::vector<std::pair<float, float>> uvs;
  std::vector<SubGeometry> geos;
  std::vector<std::string> mtl_files;
  auto model = std::make_unique<Model>();
  model->texcoords = texcoords;
  if (!ParseOBJ(obj_path, &vertices, &uvs, &geos, &mtl_files, &model->faces_dropped, err)) return nullptr;
  const auto slash = obj_path.find_last_of('/');
  const std::string folder = slash == std::string::npos ? std::string("./") : obj_path.substr(0, slash + 1);
  std::vector<std::string> names;
  for (const auto& f : mtl_files) ParseMTL(folder, f, &names, &model->materials);
  // one decoded texture per file (the reference's LoadedTextures cache, gpu_texture.h:20-28)
  for (auto& m : model->materials) {
    if (!m.use_texture) continue;
    for (size_t k = 0; k < model->textures.size(); ++k)
      if (model->textures[k].path == m.texture_path) m.texture = (int)k;
    if (m.texture < 0) {
      Texture tex;
      if (!DecodePngTexture(m.texture_path, &tex, err)) return nullptr;
      model->textures.push_back(std::move(tex));
      m.texture = (int)model->textures.size() - 1;
    }
    const Texture& tx = model->textures[m.texture];
    float rgb[3];
    TextureSample(tx.texels.data(), tx.width, tx.height, tx.channels, 0.0f, 0.0f, rgb);
    m.tex_albedo = Vec3(rgb[0], rgb[1], rgb[2]);
  }
  // per-corner vertex duplication (model_loader.cpp:302-331); uv stays (0,0)
  // unless texcoords (has_texcoords, never set by the reference)
  for (const auto& g : geos) {
    uint32_t mat = 0;
    for (size_t k = 0; k < names.size(); ++k)
      if (names[k] == g.material) { mat = static_cast<uint32_t>(k); break; }
    for (const auto& f : g.faces) {
      Triangle t;
      t.material_idx = mat;
      for (int c = 0; c < 3; ++c) {
        if (f.v[c] >= vertices.size()) {
          *err = "face references vertex " + std::to_string(f.v[c] + 1) + " out of range";
          return nullptr;
        }
        const Vec3& p = vertices[f.v[c]];
        srt_vertex sv{};
        sv.vertex[0] = p.x; sv.vertex[1] = p.y; sv.vertex[2] = p.z;
        if (texcoords && f.t_ok) {
          if (f.t[c] >= uvs.size()) {
            *err = "face references texcoord " + std::to_string(f.t[c] + 1) + " out of range";
            return nullptr;
          }
          sv.texture[0] = uvs[f.t[c]].first;
          sv.texture[1] = uvs[f.t[c]].second;
        }
        model->vertices.push_back(sv);
        t.vertex_idxs[c] = static_cast<uint32_t>(model->vertices.size() - 1);
      }
      model->prims.push_back(t);
    }
  }
  if (model->prims.empty()) {
    *err = "no triangles in " + obj_path;
    return nullptr;
  }
  BuildBVH(model.get());
  return model;
}

std::unique_ptr<Model> ModelFromTriangles(const float* xyz9, uint32_t n, const Vec3& kd, const Vec3& ks,
                                          float ns) {
  auto model = std::make_unique<Model>();
  Material m;
  m.diffuse = kd;
  m.specular = ks;
  m.specular_ex = ns;
  model->materials.push_back(m);
  model->vertices.resize(size_t(n) * 3);
  model->prims.resize(n);
  for (uint32_t t = 0; t < n; ++t) {
    for (int c = 0; c < 3; ++c) {
      srt_vertex& sv = model->vertices[size_t(t) * 3 + c];
      sv = srt_vertex{};
      sv.vertex[0] = xyz9[size_t(t) * 9 + c * 3 + 0];
      sv.vertex[1] = xyz9[size_t(t) * 9 + c * 3 + 1];
      sv.vertex[2] = xyz9[size_t(t) * 9 + c * 3 + 2];
      model->prims[t].vertex_idxs[c] = t * 3 + c;
    }
    model->prims[t].material_idx = 0;
  }
  if (n > 0) BuildBVH(model.get());
  return model;
}

// gpu_loader.cpp:63-133 (the index rebasing; uploads happen in the context)
std::unique_ptr<Scene> FlattenModels(const std::vector<const Model*>& models, std::string* err) {
  auto s = std::make_unique<Scene>();
  uint32_t node_off = 0, tri_off = 0, mat_off = 0, vert_off = 0;
  for (const Model* m : models) {
    if (!m) {
      *err = "Model was null!";
      return nullptr;
    }
    const uint32_t model_mat_off = mat_off;
    const uint32_t model_tex_off = static_cast<uint32_t>(s->textures.size());
    s->textures.insert(s->textures.end(), m->textures.begin(), m->textures.end());
    s->sample_textures = s->sample_textures || (m->texcoords && !m->textures.empty());
    for (const auto& mat : m->materials) {
      srt_material_obj g{};
      g.diffuse[0] = mat.diffuse.x; g.diffuse[1] = mat.diffuse.y; g.diffuse[2] = mat.diffuse.z;
      g.specular[0] = mat.specular.x; g.specular[1] = mat.specular.y; g.specular[2] = mat.specular.z;
      g.specular_ex = mat.specular_ex;
      g.use_texture = mat.use_texture ? 1u : 0u;
      if (mat.use_texture) g.handle[0] = model_tex_off + static_cast<uint32_t>(mat.texture);
      s->mats.push_back(g);
      s->tex_albedo.push_back(mat.tex_albedo.x);
      s->tex_albedo.push_back(mat.tex_albedo.y);
      s->tex_albedo.push_back(mat.tex_albedo.z);
    }
    mat_off += static_cast<uint32_t>(m->materials.size());
    const uint32_t model_vert_off = vert_off;
    s->verts.insert(s->verts.end(), m->vertices.begin(), m->vertices.end());
    vert_off += static_cast<uint32_t>(m->vertices.size());
    srt_bvh_record b{};
    b.first_index = node_off;
    b.count = static_cast<uint32_t>(m->nodes.size());
    for (int i = 0; i < 16; ++i) b.frame[i] = (i % 5 == 0) ? 1.0f : 0.0f;  // glm::mat4(1)
    s->bvhs.push_back(b);
    const uint32_t local_tri_off = tri_off;
    for (const auto& t : m->prims) {
      srt_triangle g;
      g.v0_idx = t.vertex_idxs[0] + model_vert_off;
      g.v1_idx = t.vertex_idxs[1] + model_vert_off;
      g.v2_idx = t.vertex_idxs[2] + model_vert_off;
      g.material_idx = t.material_idx + model_mat_off;
      s->tris.push_back(g);
    }
    for (size_t i = 0; i < m->prims.size(); ++i)
      s->tri_input.push_back(local_tri_off + (i < m->prim_input.size() ? m->prim_input[i] : (uint32_t)i));
    tri_off += static_cast<uint32_t>(m->prims.size());
    for (const auto& n : m->nodes) {
      srt_bvh_node g;
      g.min_bounds[0] = n.min_bounds.x; g.min_bounds[1] = n.min_bounds.y; g.min_bounds[2] = n.min_bounds.z;
      g.max_bounds[0] = n.max_bounds.x; g.max_bounds[1] = n.max_bounds.y; g.max_bounds[2] = n.max_bounds.z;
      g.first_child_or_prim_index = n.prim_count > 0 ? n.first_prim_index + local_tri_off : n.first_child + node_off;
      g.prim_count = n.prim_count;
      s->nodes.push_back(g);
    }
    node_off += b.count;
  }
  return s;
}

}  // namespace srt
