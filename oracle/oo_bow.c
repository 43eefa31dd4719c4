/*
 * oracle/oo_bow.c -- TEST INFRASTRUCTURE ONLY (CPU oracle; never linked into the product).
 *
 * Restatement of Frame::ComputeBoW (src/Frame.cc:395-402) = ORBVocabulary::transform(features, mBowVec,
 * mFeatVec, 4), i.e. DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB> from
 * Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:
 *   loadFromTextFile :1338-1420   (node ids in file order, leaves numbered as words in file order)
 *   transform(features, v, fv, levelsup) :1127-1194
 *   transform(feature, word, weight, nid, levelsup) :1218-1256 (strict-< first minimum over children)
 * BowVector::addWeight / addIfNotExist / normalize (BowVector.cpp:34-84), FeatureVector::addFeature
 * (FeatureVector.cpp:31-45), FORB::distance (FORB.cpp:81-101), ScoringObject.h:74-89 (mustNormalize).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

struct oo_vocab {
    int k, L, scoring, weighting;
    int n;               /* nodes incl. the root (id 0) */
    int* parent;
    int* child_start;    /* CSR over children in insertion order */
    int* child_cnt;
    int* children;
    int* word_id;        /* -1 for non-leaves */
    double* weight;
    uint8_t* desc;       /* n x 32 */
    int nwords;
};

static oo_vocab* oo_vocab_build(int k, int L, int scoring, int weighting, int nn, const int* parent,
                                const uint8_t* is_leaf, const uint8_t* desc, const double* weight)
{
    /* nn entries describe nodes 1..nn (node 0 = root) exactly as the text file lists them */
    oo_vocab* v = (oo_vocab*)calloc(1, sizeof(oo_vocab));
    v->k = k; v->L = L; v->scoring = scoring; v->weighting = weighting;
    v->n = nn + 1;
    v->parent = (int*)calloc((size_t)v->n, sizeof(int));
    v->child_start = (int*)calloc((size_t)v->n + 1, sizeof(int));
    v->child_cnt = (int*)calloc((size_t)v->n, sizeof(int));
    v->children = (int*)calloc((size_t)v->n, sizeof(int));
    v->word_id = (int*)malloc(sizeof(int) * (size_t)v->n);
    v->weight = (double*)calloc((size_t)v->n, sizeof(double));
    v->desc = (uint8_t*)calloc((size_t)v->n, 32);
    v->word_id[0] = -1;
    for (int i = 0; i < nn; i++) {
        const int id = i + 1;
        v->parent[id] = parent[i];
        v->child_cnt[parent[i]]++;
        memcpy(v->desc + 32 * (size_t)id, desc + 32 * (size_t)i, 32);
        v->weight[id] = weight[i];
        v->word_id[id] = is_leaf[i] ? v->nwords++ : -1;
    }
    for (int i = 0; i < v->n; i++) v->child_start[i + 1] = v->child_start[i] + v->child_cnt[i];
    int* fill = (int*)calloc((size_t)v->n, sizeof(int));
    for (int id = 1; id < v->n; id++) {  /* m_nodes[pid].children.push_back(nid) in file order */
        const int p = v->parent[id];
        v->children[v->child_start[p] + fill[p]++] = id;
    }
    free(fill);
    return v;
}

oo_vocab* oo_vocab_from_arrays(int k, int L, int scoring, int weighting, int nn, const int* parent,
                               const uint8_t* is_leaf, const uint8_t* desc, const double* weight)
{
    return oo_vocab_build(k, L, scoring, weighting, nn, parent, is_leaf, desc, weight);
}

/* loadFromTextFile: "k L scoring weighting" then one line per node "pid isLeaf d0 .. d31 weight".
 * Blank lines are skipped (the reference's eof loop would parse them as a node with an undefined parent). */
oo_vocab* oo_vocab_load_text(const char* path)
{
    FILE* fp = fopen(path, "r");
    if (!fp) return NULL;
    int k, L, sc, wt;
    if (fscanf(fp, "%d %d %d %d", &k, &L, &sc, &wt) != 4) { fclose(fp); return NULL; }
    if (k < 0 || k > 20 || L < 1 || L > 10 || sc < 0 || sc > 5 || wt < 0 || wt > 3) { fclose(fp); return NULL; }
    int cap = 1024, nn = 0;
    int* par = (int*)malloc(sizeof(int) * cap);
    uint8_t* leaf = (uint8_t*)malloc((size_t)cap);
    uint8_t* desc = (uint8_t*)malloc(32 * (size_t)cap);
    double* w = (double*)malloc(sizeof(double) * cap);
    for (;;) {
        int pid, il;
        if (fscanf(fp, "%d %d", &pid, &il) != 2) break;
        if (nn == cap) {
            cap *= 2;
            par = (int*)realloc(par, sizeof(int) * cap);
            leaf = (uint8_t*)realloc(leaf, (size_t)cap);
            desc = (uint8_t*)realloc(desc, 32 * (size_t)cap);
            w = (double*)realloc(w, sizeof(double) * cap);
        }
        for (int d = 0; d < 32; d++) {
            int x;
            if (fscanf(fp, "%d", &x) != 1) x = 0;
            desc[32 * (size_t)nn + d] = (uint8_t)x;
        }
        if (fscanf(fp, "%lf", &w[nn]) != 1) w[nn] = 0;
        par[nn] = pid;
        leaf[nn] = il > 0;
        if (pid < 0 || pid > nn) { nn = -1; break; }
        nn++;
    }
    fclose(fp);
    oo_vocab* v = nn < 0 ? NULL : oo_vocab_build(k, L, sc, wt, nn, par, leaf, desc, w);
    free(par); free(leaf); free(desc); free(w);
    return v;
}

void oo_vocab_free(oo_vocab* v)
{
    if (!v) return;
    free(v->parent); free(v->child_start); free(v->child_cnt); free(v->children);
    free(v->word_id); free(v->weight); free(v->desc); free(v);
}

int oo_vocab_nodes(const oo_vocab* v) { return v->n; }
int oo_vocab_words(const oo_vocab* v) { return v->nwords; }

/* transform(feature, word_id, weight, nid, levelsup), :1218-1256 */
static void oo_transform_one(const oo_vocab* v, const uint8_t* f, int levelsup, int* word, double* weight, int* nid)
{
    const int nid_level = v->L - levelsup;
    *nid = 0;  /* root when nid_level <= 0; the reference leaves it unset if a leaf is reached earlier */
    int final_id = 0, level = 0;
    do {
        ++level;
        const int* ch = v->children + v->child_start[final_id];
        const int nc = v->child_cnt[final_id];
        final_id = ch[0];
        int best = oo_descriptor_distance(f, v->desc + 32 * (size_t)final_id);
        for (int c = 1; c < nc; c++) {
            const int d = oo_descriptor_distance(f, v->desc + 32 * (size_t)ch[c]);
            if (d < best) { best = d; final_id = ch[c]; }
        }
        if (level == nid_level) *nid = final_id;
    } while (v->child_cnt[final_id] > 0);
    *word = v->word_id[final_id];
    *weight = v->weight[final_id];
}

typedef struct { int key; int idx; } oo_pair2;
static int oo_pair2_cmp(const void* a, const void* b)
{
    const oo_pair2 *x = (const oo_pair2*)a, *y = (const oo_pair2*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* transform(features, v, fv, levelsup), :1127-1194.  Outputs: the BowVector as (word ascending, value)
 * and the FeatureVector as (node ascending, CSR of feature indices in feature order).  Returns 0. */
int oo_bow_transform(const oo_vocab* v, const uint8_t* desc, int n, int levelsup, int* words, double* values,
                     int* nwords, int* nodes, int* node_off, int* feat_idx, int* nnodes)
{
    *nwords = 0;
    *nnodes = 0;
    node_off[0] = 0;
    if (v->n <= 1) return 0;  /* empty() */
    oo_pair2* wp = (oo_pair2*)malloc(sizeof(oo_pair2) * (size_t)(n + 1));
    oo_pair2* np = (oo_pair2*)malloc(sizeof(oo_pair2) * (size_t)(n + 1));
    double* wv = (double*)malloc(sizeof(double) * (size_t)(n + 1));
    int m = 0;
    for (int i = 0; i < n; i++) {
        int w, nid;
        double wt;
        oo_transform_one(v, desc + 32 * (size_t)i, levelsup, &w, &wt, &nid);
        if (wt > 0) {  /* not stopped */
            wp[m].key = w; wp[m].idx = i; wv[i] = wt;
            np[m].key = nid; np[m].idx = i;
            m++;
        }
    }
    qsort(wp, (size_t)m, sizeof(oo_pair2), oo_pair2_cmp);
    qsort(np, (size_t)m, sizeof(oo_pair2), oo_pair2_cmp);
    const int tf = v->weighting == 0 || v->weighting == 1;  /* TF_IDF, TF: addWeight; IDF, BINARY: addIfNotExist */
    int nw = 0;
    for (int j = 0; j < m; j++) {
        if (nw > 0 && words[nw - 1] == wp[j].key) {
            if (tf) values[nw - 1] += wv[wp[j].idx];
        } else {
            words[nw] = wp[j].key;
            values[nw] = wv[wp[j].idx];
            nw++;
        }
    }
    /* mustNormalize: L1 for L1/CHI_SQUARE/KL/BHATTACHARYYA, L2 for L2_NORM, none for DOT_PRODUCT */
    const int must = v->scoring != 5;
    if (tf && nw > 0 && !must) {
        const double nd = nw;
        for (int j = 0; j < nw; j++) values[j] /= nd;
    }
    if (must) {
        double norm = 0.0;
        if (v->scoring == 1) {
            for (int j = 0; j < nw; j++) norm += values[j] * values[j];
            norm = sqrt(norm);
        } else {
            for (int j = 0; j < nw; j++) norm += fabs(values[j]);
        }
        if (norm > 0.0)
            for (int j = 0; j < nw; j++) values[j] /= norm;
    }
    int nn = 0;
    for (int j = 0; j < m; j++) {
        if (nn == 0 || nodes[nn - 1] != np[j].key) {
            nodes[nn] = np[j].key;
            node_off[nn] = j;
            nn++;
        }
        feat_idx[j] = np[j].idx;
    }
    node_off[nn] = m;
    *nwords = nw;
    *nnodes = nn;
    free(wp); free(np); free(wv);
    return 0;
}
