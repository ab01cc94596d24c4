// oni355 CPU variational-EM LDA -- the oni-lda-c equivalent.
//
// Same algorithm family as Blei's lda-c `lda est` / `lda inf` (mean-field E-step with digamma /
// log-sum-exp φ updates, closed-form β M-step, Newton update of a symmetric α) and the same file
// formats, re-implemented from the published algorithm (Blei, Ng & Jordan 2003). The reference
// fork spread documents over MPI ranks and reduced the K×V sufficient statistics per EM
// iteration; here documents are spread over OpenMP threads with thread-private statistics that
// are summed in a fixed order (deterministic for a given thread count).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace oni_lda {

struct Settings {
  int var_max_iter = 20;
  double var_convergence = 1e-6;
  int em_max_iter = 100;
  double em_convergence = 1e-4;
  bool estimate_alpha = true;
  int lag = 5;            // snapshot NNN.* every `lag` EM iterations (0 = never)
  uint64_t seed = 4357;   // init RNG (lda-c used a time-seeded MT19937)
  int threads = 0;        // 0 = OpenMP default
};

struct Corpus {
  int num_terms = 0;
  std::vector<int64_t> doc_ptr;  // [D+1] into words/counts
  std::vector<int32_t> words;
  std::vector<int32_t> counts;
  int num_docs() const { return (int)doc_ptr.size() - 1; }
  int64_t total(int d) const;
};

struct Model {
  int K = 0, V = 0;
  double alpha = 0;
  std::vector<double> log_prob_w;  // [K][V]
};

struct EmResult {
  std::vector<double> gamma;      // [D][K]
  std::vector<double> likelihood; // per EM iteration
  std::vector<double> convergence;
  std::vector<int> argmax_topic;  // per (doc, unique word) in corpus order: word-assignments.dat
  int iterations = 0;
};

bool read_settings(const std::string& path, Settings* s, std::string* err);
bool read_corpus(const std::string& path, Corpus* c, std::string* err);
bool save_model(const Model& m, const std::string& prefix, std::string* err);
bool load_model(const std::string& prefix, Model* m, std::string* err);
bool save_gamma(const std::vector<double>& gamma, int D, int K, const std::string& path);

// init: "random", "seeded", or a model prefix to resume from.
EmResult run_em(const Corpus& c, Model* m, int K, double alpha, const std::string& init, const Settings& s,
                const std::string& out_dir);
// inference only (lda inf): returns per-doc likelihoods, fills gamma.
std::vector<double> infer(const Corpus& c, const Model& m, const Settings& s, std::vector<double>* gamma);

double digamma(double x);
double trigamma(double x);
double log_sum(double log_a, double log_b);

}  // namespace oni_lda
