// oni355 CPU variational-EM LDA (see lda_vem.h).
#include "lda_vem.h"

#include <omp.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>

namespace oni_lda {

// ------------------------------------------------------------------------------------------------
// special functions
// ------------------------------------------------------------------------------------------------
double digamma(double x) {
  double r = 0.0;
  while (x < 6.0) {
    r -= 1.0 / x;
    x += 1.0;
  }
  const double f = 1.0 / (x * x);
  const double t = f * (-1.0 / 12 + f * (1.0 / 120 + f * (-1.0 / 252 + f * (1.0 / 240 + f * (-1.0 / 132)))));
  return r + std::log(x) - 0.5 / x + t;
}

double trigamma(double x) {
  double r = 0.0;
  while (x < 6.0) {
    r += 1.0 / (x * x);
    x += 1.0;
  }
  const double f = 1.0 / (x * x);
  const double t = 1.0 / x + f / 2.0 + f / x * (1.0 / 6 + f * (-1.0 / 30 + f * (1.0 / 42 + f * (-1.0 / 30))));
  return r + t;
}

double log_sum(double a, double b) {
  if (a < b) std::swap(a, b);
  return a + std::log1p(std::exp(b - a));
}

int64_t Corpus::total(int d) const {
  int64_t t = 0;
  for (int64_t i = doc_ptr[d]; i < doc_ptr[d + 1]; ++i) t += counts[i];
  return t;
}

// ------------------------------------------------------------------------------------------------
// file I/O (lda-c formats)
// ------------------------------------------------------------------------------------------------
bool read_settings(const std::string& path, Settings* s, std::string* err) {
  std::ifstream f(path);
  if (!f) {
    *err = "cannot open settings " + path;
    return false;
  }
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream is(line);
    std::vector<std::string> tok;
    std::string t;
    while (is >> t) tok.push_back(t);
    if (tok.empty() || tok[0][0] == '#') continue;
    std::string key;
    for (size_t i = 0; i + 1 < tok.size(); ++i) key += (i ? " " : "") + tok[i];
    const std::string& v = tok.back();
    if (key == "var max iter") s->var_max_iter = std::stoi(v);
    else if (key == "var convergence") s->var_convergence = std::stod(v);
    else if (key == "em max iter") s->em_max_iter = std::stoi(v);
    else if (key == "em convergence") s->em_convergence = std::stod(v);
    else if (key == "alpha") s->estimate_alpha = (v == "estimate");
    else if (key == "lag") s->lag = std::stoi(v);
    else if (key == "seed") s->seed = std::stoull(v);
    else if (key == "threads") s->threads = std::stoi(v);
  }
  return true;
}

bool read_corpus(const std::string& path, Corpus* c, std::string* err) {
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) {
    *err = "cannot open corpus " + path;
    return false;
  }
  c->doc_ptr.assign(1, 0);
  c->words.clear();
  c->counts.clear();
  int max_w = -1;
  int m;
  while (std::fscanf(f, "%d", &m) == 1) {
    for (int i = 0; i < m; ++i) {
      int w, n;
      if (std::fscanf(f, "%d:%d", &w, &n) != 2 || w < 0 || n < 0) {
        std::fclose(f);
        *err = "malformed corpus line";
        return false;
      }
      c->words.push_back(w);
      c->counts.push_back(n);
      max_w = std::max(max_w, w);
    }
    c->doc_ptr.push_back((int64_t)c->words.size());
  }
  std::fclose(f);
  c->num_terms = max_w + 1;
  return true;
}

bool save_model(const Model& m, const std::string& prefix, std::string* err) {
  FILE* f = std::fopen((prefix + ".beta").c_str(), "w");
  if (!f) {
    *err = "cannot write " + prefix + ".beta";
    return false;
  }
  for (int k = 0; k < m.K; ++k) {
    for (int w = 0; w < m.V; ++w) std::fprintf(f, w ? " %5.10f" : "%5.10f", m.log_prob_w[(size_t)k * m.V + w]);
    std::fputc('\n', f);
  }
  std::fclose(f);
  f = std::fopen((prefix + ".other").c_str(), "w");
  if (!f) {
    *err = "cannot write " + prefix + ".other";
    return false;
  }
  std::fprintf(f, "num_topics %d\nnum_terms %d\nalpha %5.10f\n", m.K, m.V, m.alpha);
  std::fclose(f);
  return true;
}

bool load_model(const std::string& prefix, Model* m, std::string* err) {
  FILE* f = std::fopen((prefix + ".other").c_str(), "r");
  if (!f) {
    *err = "cannot open " + prefix + ".other";
    return false;
  }
  if (std::fscanf(f, "num_topics %d\nnum_terms %d\nalpha %lf", &m->K, &m->V, &m->alpha) != 3) {
    std::fclose(f);
    *err = "malformed .other";
    return false;
  }
  std::fclose(f);
  f = std::fopen((prefix + ".beta").c_str(), "r");
  if (!f) {
    *err = "cannot open " + prefix + ".beta";
    return false;
  }
  m->log_prob_w.assign((size_t)m->K * m->V, 0.0);
  for (size_t i = 0; i < m->log_prob_w.size(); ++i)
    if (std::fscanf(f, "%lf", &m->log_prob_w[i]) != 1) {
      std::fclose(f);
      *err = "malformed .beta";
      return false;
    }
  std::fclose(f);
  return true;
}

bool save_gamma(const std::vector<double>& gamma, int D, int K, const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) return false;
  for (int d = 0; d < D; ++d) {
    for (int k = 0; k < K; ++k) std::fprintf(f, k ? " %5.10f" : "%5.10f", gamma[(size_t)d * K + k]);
    std::fputc('\n', f);
  }
  std::fclose(f);
  return true;
}

// ------------------------------------------------------------------------------------------------
// inference
// ------------------------------------------------------------------------------------------------
namespace {

struct Stats {
  std::vector<double> class_word;  // [K][V]
  std::vector<double> class_total;  // [K]
  double alpha_ss = 0;
  int num_docs = 0;
  void init(int K, int V) {
    class_word.assign((size_t)K * V, 0.0);
    class_total.assign(K, 0.0);
    alpha_ss = 0;
    num_docs = 0;
  }
};

double doc_likelihood(const Corpus& c, int d, const Model& m, const std::vector<double>& phi,
                      const std::vector<double>& gamma, std::vector<double>& dig) {
  const int K = m.K;
  double gsum = 0;
  for (int k = 0; k < K; ++k) {
    dig[k] = digamma(gamma[k]);
    gsum += gamma[k];
  }
  const double digsum = digamma(gsum);
  double L = std::lgamma(m.alpha * K) - K * std::lgamma(m.alpha) - std::lgamma(gsum);
  const int64_t lo = c.doc_ptr[d], hi = c.doc_ptr[d + 1];
  for (int k = 0; k < K; ++k) {
    const double e = dig[k] - digsum;
    L += (m.alpha - 1) * e + std::lgamma(gamma[k]) - (gamma[k] - 1) * e;
    for (int64_t i = lo; i < hi; ++i) {
      const double p = phi[(size_t)(i - lo) * K + k];
      if (p > 0) L += c.counts[i] * p * (e - std::log(p) + m.log_prob_w[(size_t)k * m.V + c.words[i]]);
    }
  }
  return L;
}

// Mean-field E-step for one document; phi is [n_unique][K], gamma [K].
double infer_doc(const Corpus& c, int d, const Model& m, int var_max_iter, double var_conv, std::vector<double>& phi,
                 std::vector<double>& gamma, std::vector<double>& dig, std::vector<double>& old) {
  const int K = m.K;
  const int64_t lo = c.doc_ptr[d], hi = c.doc_ptr[d + 1];
  const int64_t n = hi - lo;
  const double tot = (double)c.total(d);
  phi.assign((size_t)n * K, 1.0 / K);
  for (int k = 0; k < K; ++k) {
    gamma[k] = m.alpha + tot / K;
    dig[k] = digamma(gamma[k]);
  }
  double L_old = 0, L = 0, conv = 1;
  for (int it = 0; conv > var_conv && (it < var_max_iter || var_max_iter == -1); ++it) {
    for (int64_t i = 0; i < n; ++i) {
      const int w = c.words[lo + i];
      const double cnt = c.counts[lo + i];
      double* ph = &phi[(size_t)i * K];
      double s = 0;
      for (int k = 0; k < K; ++k) {
        old[k] = ph[k];
        ph[k] = dig[k] + m.log_prob_w[(size_t)k * m.V + w];
        s = k ? log_sum(s, ph[k]) : ph[k];
      }
      for (int k = 0; k < K; ++k) {
        ph[k] = std::exp(ph[k] - s);
        gamma[k] += cnt * (ph[k] - old[k]);
        dig[k] = digamma(gamma[k]);
      }
    }
    L = doc_likelihood(c, d, m, phi, gamma, dig);
    conv = (L_old == 0) ? 1.0 : (L_old - L) / L_old;
    L_old = L;
  }
  return L;
}

void mle(Model* m, const Stats& ss, bool est_alpha) {
  const int K = m->K, V = m->V;
  for (int k = 0; k < K; ++k)
    for (int w = 0; w < V; ++w) {
      const double cw = ss.class_word[(size_t)k * V + w];
      m->log_prob_w[(size_t)k * V + w] = cw > 0 ? std::log(cw) - std::log(ss.class_total[k]) : -100.0;
    }
  if (est_alpha && ss.num_docs > 0) {
    // Newton's method on log(alpha) for the symmetric Dirichlet
    const double D = ss.num_docs;
    double init_a = 100.0, log_a = std::log(init_a), df = 1;
    for (int it = 0; it < 1000 && std::fabs(df) > 1e-5; ++it) {
      double a = std::exp(log_a);
      if (std::isnan(a)) {
        init_a *= 10;
        a = init_a;
        log_a = std::log(a);
      }
      df = D * (K * digamma(K * a) - K * digamma(a)) + ss.alpha_ss;
      const double d2f = D * (K * K * trigamma(K * a) - K * trigamma(a));
      log_a -= df / (d2f * a + df);
    }
    m->alpha = std::exp(log_a);
  }
}

// E-step over all docs with thread-private statistics (static partition → deterministic).
double e_step(const Corpus& c, const Model& m, int var_max_iter, double var_conv, Stats* total,
              std::vector<double>* gamma_all, int threads) {
  const int D = c.num_docs(), K = m.K, V = m.V;
  const int nt = threads > 0 ? threads : omp_get_max_threads();
  std::vector<Stats> loc(nt);
  std::vector<double> lik(nt, 0.0);
#pragma omp parallel num_threads(nt)
  {
    const int t = omp_get_thread_num();
    Stats& ss = loc[t];
    ss.init(K, V);
    std::vector<double> phi, gamma(K), dig(K), old(K);
#pragma omp for schedule(static)
    for (int d = 0; d < D; ++d) {
      lik[t] += infer_doc(c, d, m, var_max_iter, var_conv, phi, gamma, dig, old);
      double gsum = 0;
      for (int k = 0; k < K; ++k) {
        gsum += gamma[k];
        ss.alpha_ss += digamma(gamma[k]);
      }
      ss.alpha_ss -= K * digamma(gsum);
      const int64_t lo = c.doc_ptr[d];
      for (int64_t i = lo; i < c.doc_ptr[d + 1]; ++i)
        for (int k = 0; k < K; ++k) {
          const double v = c.counts[i] * phi[(size_t)(i - lo) * K + k];
          ss.class_word[(size_t)k * V + c.words[i]] += v;
          ss.class_total[k] += v;
        }
      ss.num_docs++;
      if (gamma_all) std::copy(gamma.begin(), gamma.end(), gamma_all->begin() + (size_t)d * K);
    }
  }
  total->init(K, V);
  double L = 0;
  for (int t = 0; t < nt; ++t) {
    for (size_t i = 0; i < total->class_word.size(); ++i) total->class_word[i] += loc[t].class_word[i];
    for (int k = 0; k < K; ++k) total->class_total[k] += loc[t].class_total[k];
    total->alpha_ss += loc[t].alpha_ss;
    total->num_docs += loc[t].num_docs;
    L += lik[t];
  }
  return L;
}

}  // namespace

std::vector<double> infer(const Corpus& c, const Model& m, const Settings& s, std::vector<double>* gamma) {
  const int D = c.num_docs(), K = m.K;
  gamma->assign((size_t)D * K, 0.0);
  std::vector<double> lik(D);
  const int nt = s.threads > 0 ? s.threads : omp_get_max_threads();
#pragma omp parallel num_threads(nt)
  {
    std::vector<double> phi, g(K), dig(K), old(K);
#pragma omp for schedule(dynamic, 16)
    for (int d = 0; d < D; ++d) {
      lik[d] = infer_doc(c, d, m, s.var_max_iter, s.var_convergence, phi, g, dig, old);
      std::copy(g.begin(), g.end(), gamma->begin() + (size_t)d * K);
    }
  }
  return lik;
}

EmResult run_em(const Corpus& c, Model* m, int K, double alpha, const std::string& init, const Settings& s,
                const std::string& out_dir) {
  EmResult r;
  const int D = c.num_docs();
  std::string err;
  Stats ss;
  if (init == "random" || init == "seeded") {
    m->K = K;
    m->V = c.num_terms;
    m->alpha = alpha;
    m->log_prob_w.assign((size_t)K * m->V, 0.0);
    ss.init(K, m->V);
    std::mt19937_64 rng(s.seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    if (init == "random") {
      for (int k = 0; k < K; ++k)
        for (int w = 0; w < m->V; ++w) {
          const double v = 1.0 / m->V + U(rng);
          ss.class_word[(size_t)k * m->V + w] = v;
          ss.class_total[k] += v;
        }
    } else {
      std::uniform_int_distribution<int> pick(0, std::max(D - 1, 0));
      for (int k = 0; k < K; ++k) {
        const int d = pick(rng);
        for (int64_t i = c.doc_ptr[d]; i < c.doc_ptr[d + 1]; ++i)
          ss.class_word[(size_t)k * m->V + c.words[i]] += c.counts[i];
        for (int w = 0; w < m->V; ++w) {
          ss.class_word[(size_t)k * m->V + w] += 1.0;
          ss.class_total[k] += ss.class_word[(size_t)k * m->V + w];
        }
      }
    }
    mle(m, ss, false);
  } else if (!load_model(init, m, &err)) {
    std::fprintf(stderr, "lda: %s\n", err.c_str());
    return r;
  }
  FILE* lf = out_dir.empty() ? nullptr : std::fopen((out_dir + "/likelihood.dat").c_str(), "w");
  int var_max_iter = s.var_max_iter;
  double L_old = 0, conv = 1;
  int i = 0;
  while (((conv < 0) || (conv > s.em_convergence) || (i <= 2)) && (i <= s.em_max_iter)) {
    ++i;
    const double L = e_step(c, *m, var_max_iter, s.var_convergence, &ss, nullptr, s.threads);
    mle(m, ss, s.estimate_alpha);
    conv = (L_old == 0) ? 1.0 : (L_old - L) / L_old;
    if (conv < 0) var_max_iter *= 2;
    L_old = L;
    r.likelihood.push_back(L);
    r.convergence.push_back(conv);
    if (lf) {
      std::fprintf(lf, "%10.10f\t%5.5e\n", L, conv);
      std::fflush(lf);
    }
    if (!out_dir.empty() && s.lag > 0 && i % s.lag == 0) {
      char buf[32];
      std::snprintf(buf, sizeof buf, "/%03d", i);
      save_model(*m, out_dir + buf, &err);
    }
  }
  if (lf) std::fclose(lf);
  r.iterations = i;
  // final E-step: gamma + word assignments with the final model
  r.gamma.assign((size_t)D * m->K, 0.0);
  r.argmax_topic.assign(c.words.size(), 0);
  const int nt = s.threads > 0 ? s.threads : omp_get_max_threads();
#pragma omp parallel num_threads(nt)
  {
    std::vector<double> phi, g(m->K), dig(m->K), old(m->K);
#pragma omp for schedule(dynamic, 16)
    for (int d = 0; d < D; ++d) {
      infer_doc(c, d, *m, var_max_iter, s.var_convergence, phi, g, dig, old);
      std::copy(g.begin(), g.end(), r.gamma.begin() + (size_t)d * m->K);
      const int64_t lo = c.doc_ptr[d];
      for (int64_t i2 = lo; i2 < c.doc_ptr[d + 1]; ++i2) {
        const double* ph = &phi[(size_t)(i2 - lo) * m->K];
        r.argmax_topic[i2] = (int)(std::max_element(ph, ph + m->K) - ph);
      }
    }
  }
  if (!out_dir.empty()) {
    save_model(*m, out_dir + "/final", &err);
    save_gamma(r.gamma, D, m->K, out_dir + "/final.gamma");
    FILE* wa = std::fopen((out_dir + "/word-assignments.dat").c_str(), "w");
    if (wa) {
      for (int d = 0; d < D; ++d) {
        std::fprintf(wa, "%03d", (int)(c.doc_ptr[d + 1] - c.doc_ptr[d]));
        for (int64_t i2 = c.doc_ptr[d]; i2 < c.doc_ptr[d + 1]; ++i2)
          std::fprintf(wa, " %04d:%02d", c.words[i2], r.argmax_topic[i2]);
        std::fputc('\n', wa);
      }
      std::fclose(wa);
    }
  }
  return r;
}

}  // namespace oni_lda

// ------------------------------------------------------------------------------------------------
// C ABI for ctypes (oni355/models/vem.py)
// ------------------------------------------------------------------------------------------------
#include "../native/oni_native.h"

ONI_NATIVE_API int oni_vem_est(const int64_t* doc_ptr, const int32_t* words, const int32_t* counts, int D, int V,
                               int K, double alpha, int estimate_alpha, int var_max_iter, double var_conv,
                               int em_max_iter, double em_conv, uint64_t seed, int seeded_init, int threads,
                               double* out_log_beta, double* out_gamma, double* out_alpha, double* out_lik,
                               int* out_iters) {
  oni_lda::Corpus c;
  c.num_terms = V;
  c.doc_ptr.assign(doc_ptr, doc_ptr + D + 1);
  c.words.assign(words, words + doc_ptr[D]);
  c.counts.assign(counts, counts + doc_ptr[D]);
  oni_lda::Settings s;
  s.var_max_iter = var_max_iter;
  s.var_convergence = var_conv;
  s.em_max_iter = em_max_iter;
  s.em_convergence = em_conv;
  s.estimate_alpha = estimate_alpha != 0;
  s.seed = seed;
  s.threads = threads;
  s.lag = 0;
  oni_lda::Model m;
  auto r = oni_lda::run_em(c, &m, K, alpha, seeded_init ? "seeded" : "random", s, "");
  if (m.log_prob_w.size() != (size_t)K * V) return 1;
  std::memcpy(out_log_beta, m.log_prob_w.data(), sizeof(double) * K * V);
  std::memcpy(out_gamma, r.gamma.data(), sizeof(double) * (size_t)D * K);
  *out_alpha = m.alpha;
  for (size_t i = 0; i < r.likelihood.size() && (int)i <= em_max_iter; ++i) out_lik[i] = r.likelihood[i];
  *out_iters = r.iterations;
  return 0;
}
