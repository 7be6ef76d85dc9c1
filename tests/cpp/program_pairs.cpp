// Structural check of the threaded program's paired BVH steps (compile.cpp), host only:
//   program_pairs <scene.json> <expect_pairs 0|1>
// For every BVH / accelerated-list tree step of the wide program: word 2 is the step after a hit
// and word 3 the step after a hit whose paired box misses. A paired step (word 2 != i + 1) must
// sit right before a step of its own kind (its near child), carry that child's box in words 7,
// 11-15 and the child's skip index in word 3, and no skip index of any step may land on the
// child (so the child's step is never reached). Prints "pairs=<n> steps=<n>" and exits non-zero
// on the first violation.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "scene.h"

using namespace rt2;

static int fail(const char* what, size_t i) {
  std::fprintf(stderr, "violation at step %zu: %s\n", i, what);
  return 1;
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  Scene s;
  std::string err;
  if (!LoadScene(argv[1], 0x5EED2024ull, s, err)) {
    std::fprintf(stderr, "load: %s\n", err.c_str());
    return 2;
  }
  CompiledScene c;
  if (!CompileScene(s, c, err)) {
    std::fprintf(stderr, "compile: %s\n", err.c_str());
    return 2;
  }
  const size_t n = c.lin.size() / 4;
  if (n == 0 || c.lin_wide.size() != 16 * (n + 1)) return fail("no wide program", 0);
  if (c.lin_wide[16 * n] != kProgramEnd) return fail("no kProgramEnd entry after the last step", n);
  std::vector<char> target(n + 1, 0), second(n + 1, 0);
  for (size_t i = 0; i < n; i++) {
    const uint32_t k = c.lin[4 * i];
    if (k == kBvh || k == kAccBvh) target[c.lin[4 * i + 1]] = 1;
  }
  size_t pairs = 0;
  for (size_t i = 0; i < n; i++) {
    const uint32_t k = c.lin[4 * i];
    if (k != kBvh && k != kAccBvh) continue;
    const uint32_t* w = &c.lin_wide[16 * i];
    if (w[1] != c.lin[4 * i + 1]) return fail("skip word", i);
    if (w[2] == i + 1) {
      if (w[3] != c.lin[4 * i + 1]) return fail("single step: word 3 is not its skip", i);
      continue;
    }
    pairs++;
    const size_t ch = i + 1;
    if (ch >= n || c.lin[4 * ch] != k) return fail("paired step not followed by its kind", i);
    if (w[2] != ch + 1) return fail("word 2 is not past the child", i);
    if (w[3] != c.lin[4 * ch + 1]) return fail("word 3 is not the child's skip", i);
    if (target[ch]) return fail("a skip index lands on the paired child", i);
    if (second[i]) return fail("a paired child is itself paired", i);
    second[ch] = 1;
    const float* b = &c.lind[4 * (size_t)c.lin[4 * ch + 2]];
    const int words[6] = {7, 11, 12, 13, 14, 15}, rec[6] = {0, 1, 2, 4, 5, 6};
    for (int j = 0; j < 6; j++)
      if (std::memcmp(&w[words[j]], &b[rec[j]], 4) != 0) return fail("child box words", i);
  }
  // LISTACC steps: skip = the index after the list's tree, whose steps (and only they) lie between
  // (the kernel walks them lane by lane, render.hip)
  size_t lists = 0;
  for (size_t i = 0; i < n; i++) {
    if (c.lin[4 * i] != kListAcc) continue;
    lists++;
    const size_t end = c.lin[4 * i + 1], copy = c.lin[4 * i + 3];
    if (end <= i + 1 || end > n) return fail("LISTACC skip is not past its tree", i);
    if (copy == 0 || (end - i - 1 != copy && end - i - 1 != 8 * copy)) return fail("LISTACC copies", i);
    for (size_t j = i + 1; j < end; j++)
      if (c.lin[4 * j] != kAccBvh && c.lin[4 * j] != kAccSphere) return fail("a non-tree step inside a LISTACC tree", j);
    if (end < n && (c.lin[4 * end] == kAccBvh || c.lin[4 * end] == kAccSphere)) return fail("LISTACC skip lands in a tree", i);
    for (size_t j = i + 1; j < end; j++)
      if (c.lin[4 * j] == kAccBvh && (c.lin[4 * j + 1] <= j || c.lin[4 * j + 1] > end || c.lin_wide[16 * j + 2] > end ||
                                       c.lin_wide[16 * j + 3] > end))
        return fail("a tree step's targets leave the tree", j);
  }
  std::printf("pairs=%zu steps=%zu lists=%zu\n", pairs, n, lists);
  const bool expect = std::atoi(argv[2]) != 0;
  if (expect != (pairs > 0)) return fail(expect ? "no pairs" : "unexpected pairs", 0);
  return 0;
}
