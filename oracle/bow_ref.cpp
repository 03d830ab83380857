// oracle/bow_ref.cpp -- TEST INFRASTRUCTURE ONLY (checker; see orb_ref.cpp header).
//
// DBoW2's vocabulary as the reference uses it (see oracle_bow.h for the functions restated).

#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>

#include "oracle_bow.h"

namespace oracle {

int Vocabulary::load_text(const char* path, std::string* err) {
  std::ifstream f(path);
  if (!f.is_open()) {
    *err = std::string("cannot open vocabulary ") + path;
    return -1;
  }
  parent.clear();
  word_of.clear();
  children.clear();
  desc.clear();
  weight.clear();
  words.clear();
  std::string s;
  std::getline(f, s);
  std::stringstream ss;
  ss << s;
  int n1 = -1, n2 = -1;
  k = -1;
  L = -1;
  ss >> k;
  ss >> L;
  ss >> n1;
  ss >> n2;
  if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) {
    *err = "Vocabulary loading failure: This is not a correct text file!";
    return -1;
  }
  if (n1 > 1) {
    *err = "scoring type other than L1 / L2 norm is not restated";
    return -1;
  }
  scoring = n1;
  weighting = n2;
  // node 0: the root
  parent.push_back(-1);
  word_of.push_back(-1);
  children.emplace_back();
  desc.resize(32, 0);
  weight.push_back(0);
  std::vector<uint8_t> leafFlag{0};
  while (!f.eof()) {
    std::string snode;
    std::getline(f, snode);
    if (snode.find_first_not_of(" \t\r") == std::string::npos) continue;  // pinned (header)
    std::stringstream ssnode;
    ssnode << snode;
    const int nid = (int)parent.size();
    int pid = -1;
    ssnode >> pid;
    if (pid < 0 || pid >= nid) {
      *err = "vocabulary node " + std::to_string(nid) + ": bad parent";
      return -1;
    }
    parent.push_back(pid);
    children[pid].push_back(nid);
    children.emplace_back();
    int nIsLeaf = 0;
    ssnode >> nIsLeaf;
    std::stringstream ssd;
    for (int iD = 0; iD < 32; iD++) {
      std::string sElement;
      ssnode >> sElement;
      ssd << sElement << " ";
    }
    // FORB::fromString (FORB.cpp): a byte is written only when its integer parses
    uint8_t d[32] = {0};
    {
      std::stringstream sd(ssd.str());
      for (int i = 0; i < 32; i++) {
        int n;
        sd >> n;
        if (!sd.fail()) d[i] = (uint8_t)n;
      }
    }
    desc.insert(desc.end(), d, d + 32);
    double w = 0;
    ssnode >> w;
    weight.push_back(w);
    leafFlag.push_back(nIsLeaf > 0);
    if (nIsLeaf > 0) {
      word_of.push_back((int)words.size());
      words.push_back(nid);
    } else {
      word_of.push_back(-1);
    }
  }
  // transform stops at a node without children (Node::isLeaf) and reads its word id: a node
  // without children must be a word, and a word must have no children
  for (size_t n = 1; n < parent.size(); n++)
    if (children[n].empty() != (leafFlag[n] != 0)) {
      *err = "vocabulary node " + std::to_string(n) + ": leaf flag and children disagree";
      return -1;
    }
  return 0;
}

void Vocabulary::transform1(const uint8_t* d, int levelsup, uint32_t& word, double& w,
                            uint32_t& nid) const {
  const int nid_level = L - levelsup;
  if (nid_level <= 0) nid = 0;
  int final_id = 0, current_level = 0;
  do {
    ++current_level;
    const std::vector<int>& nodes = children[final_id];
    final_id = nodes[0];
    int best_d = descriptor_distance(d, &desc[32 * (size_t)final_id]);
    for (size_t c = 1; c < nodes.size(); c++) {
      const int dd = descriptor_distance(d, &desc[32 * (size_t)nodes[c]]);
      if (dd < best_d) {
        best_d = dd;
        final_id = nodes[c];
      }
    }
    if (current_level == nid_level) nid = (uint32_t)final_id;
  } while (!children[final_id].empty());
  word = (uint32_t)word_of[final_id];
  w = weight[final_id];
}

void Vocabulary::transform(const uint8_t* ds, int n, int levelsup, BowVec& v, FeatVecO& fv) const {
  v = BowVec();
  fv = FeatVecO();
  if (empty()) return;
  // every scoring restated here normalises (L1 or L2); DotProduct would not
  const bool must = true;
  const bool l1 = scoring != 1;
  // std::map semantics on flat arrays: insertion keeps the word / node order
  auto bow_find = [&](uint32_t id) {
    return (size_t)(std::lower_bound(v.word.begin(), v.word.end(), id) - v.word.begin());
  };
  std::vector<std::vector<int>> fl;  // features per node, parallel to fv.node
  const bool add = weighting == 0 || weighting == 1;  // TF_IDF, TF: addWeight; IDF, BINARY: addIfNotExist
  for (int i = 0; i < n; i++) {
    uint32_t id = 0, nid = 0;
    double w = 0;
    transform1(ds + 32 * (size_t)i, levelsup, id, w, nid);
    if (!(w > 0)) continue;  // stopped word
    const size_t p = bow_find(id);
    if (p < v.word.size() && v.word[p] == id) {
      if (add) v.value[p] += w;
    } else {
      v.word.insert(v.word.begin() + p, id);
      v.value.insert(v.value.begin() + p, w);
    }
    const size_t q = (size_t)(std::lower_bound(fv.node.begin(), fv.node.end(), nid) - fv.node.begin());
    if (q < fv.node.size() && fv.node[q] == nid) {
      fl[q].push_back(i);
    } else {
      fv.node.insert(fv.node.begin() + q, nid);
      fl.insert(fl.begin() + q, std::vector<int>{i});
    }
  }
  (void)must;
  // BowVector::normalize (BowVector.cpp:62-84)
  double norm = 0.0;
  if (l1) {
    for (double x : v.value) norm += std::fabs(x);
  } else {
    for (double x : v.value) norm += x * x;
    norm = std::sqrt(norm);
  }
  if (norm > 0.0)
    for (double& x : v.value) x /= norm;
  fv.start.assign(1, 0);
  for (const auto& l : fl) {
    fv.feat.insert(fv.feat.end(), l.begin(), l.end());
    fv.start.push_back((int)fv.feat.size());
  }
}

double Vocabulary::score(const BowVec& a, const BowVec& b) const {
  // the iterators step over the sorted words (the lower_bound jumps land on the same entries)
  size_t i = 0, j = 0;
  double s = 0;
  if (scoring == 1) {  // L2Scoring
    while (i < a.word.size() && j < b.word.size()) {
      if (a.word[i] == b.word[j]) {
        s += a.value[i] * b.value[j];
        i++;
        j++;
      } else if (a.word[i] < b.word[j]) {
        i = (size_t)(std::lower_bound(a.word.begin(), a.word.end(), b.word[j]) - a.word.begin());
      } else {
        j = (size_t)(std::lower_bound(b.word.begin(), b.word.end(), a.word[i]) - b.word.begin());
      }
    }
    if (s >= 1) return 1.0;
    return 1.0 - std::sqrt(1.0 - s);
  }
  while (i < a.word.size() && j < b.word.size()) {  // L1Scoring (ScoringObject.cpp)
    const double vi = a.value[i], wi = b.value[j];
    if (a.word[i] == b.word[j]) {
      s += std::fabs(vi - wi) - std::fabs(vi) - std::fabs(wi);
      i++;
      j++;
    } else if (a.word[i] < b.word[j]) {
      i = (size_t)(std::lower_bound(a.word.begin(), a.word.end(), b.word[j]) - a.word.begin());
    } else {
      j = (size_t)(std::lower_bound(b.word.begin(), b.word.end(), a.word[i]) - b.word.begin());
    }
  }
  return -s / 2.0;
}

}  // namespace oracle
