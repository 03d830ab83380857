// oracle/oracle_bow.h -- TEST INFRASTRUCTURE ONLY (see orb_ref.cpp header).
//
// CPU restatement of the vocabulary-driven part of the reference's RGB-D path:
//   DBoW2 TemplatedVocabulary::loadFromTextFile  Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424
//   TemplatedVocabulary::transform (BowVector + FeatureVector, levelsup)            :1127-1259
//   BowVector::addWeight / addIfNotExist / normalize  BowVector.cpp:34-84
//   FeatureVector::addFeature                          FeatureVector.cpp:31-45
//   L1Scoring / L2Scoring::score                       ScoringObject.cpp
// The algorithm of DBoW2 is vendored in the reference (Thirdparty/DBoW2, modified FORB distance:
// FORB.cpp); its vocabulary ORBvoc.txt is not (.MISSING_LARGE_BLOBS), so the tests use the small
// vocabulary tools/make_test_vocabulary.py writes in the same text format.
// Pinned choice: the reference's `while(!f.eof())` loop reads one empty line after a trailing
// newline and links a node to an uninitialised parent (undefined); an empty line is skipped here.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "oracle_match.h"

namespace oracle {

// DBoW2::BowVector (std::map<WordId, WordValue>) as word-ascending arrays
struct BowVec {
  std::vector<uint32_t> word;
  std::vector<double> value;
  bool empty() const { return word.empty(); }
};

// DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned int>>) owned, flat
struct FeatVecO {
  std::vector<uint32_t> node;
  std::vector<int> start{0};
  std::vector<int> feat;
  bool empty() const { return node.empty(); }
  FeatVec view() const {
    FeatVec v;
    v.n_nodes = (int)node.size();
    v.node = node.data();
    v.start = start.data();
    v.feat = feat.data();
    return v;
  }
};

struct Vocabulary {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<int> parent, word_of;  // word_of: the node's word id, -1 for inner nodes
  std::vector<std::vector<int>> children;
  std::vector<uint8_t> desc;  // 32 bytes per node
  std::vector<double> weight;
  std::vector<int> words;     // word id -> node id
  // loadFromTextFile; returns 0, or -1 with *err set
  int load_text(const char* path, std::string* err);
  bool empty() const { return words.empty(); }
  // transform(feature, word_id, weight, &nid, levelsup) TemplatedVocabulary.h:1218-1259
  void transform1(const uint8_t* d, int levelsup, uint32_t& word, double& w, uint32_t& nid) const;
  // transform(features, BowVector, FeatureVector, levelsup) TemplatedVocabulary.h:1127-1194
  void transform(const uint8_t* desc, int n, int levelsup, BowVec& v, FeatVecO& fv) const;
  // score(v1, v2): L1Scoring / L2Scoring (the scorings this restatement accepts)
  double score(const BowVec& a, const BowVec& b) const;
};

}  // namespace oracle
