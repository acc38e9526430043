// adapter_test.cpp — compiles the ggml-backend adapter core (adapter/mi355x_ggml_mirror.hpp)
// against include/ggml_mi355x.h and runs its mirror + lowering on a graph of ggml_tensor
// structs (test infrastructure, driven by tests/test_adapter.py; host only, no device).
//
// `struct ggml_tensor` below has the fields and array sizes of upstream ggml.h [U]
// (GGML_MAX_DIMS 4, GGML_MAX_SRC 10, GGML_MAX_OP_PARAMS 64 bytes, GGML_MAX_NAME 64,
// GGML_TENSOR_FLAG_OUTPUT 2) — the members the adapter reads, with ggml's names, so the
// template instantiates exactly as it does on `struct ggml_tensor` in llama.cpp's tree.
// The op is kept as its ggml_op_name() string (the enum values differ between versions).
//
// input (argv[1]): one line per tensor
//   T id type op_name ne0..3 nb0..3 op_params[16] flags src[10] view_src view_offs data name
// (ids, -1 = null; name "-" = empty), then "N n id0 id1 ..." (the cgraph's nodes).
// argv[2..5]: cells_eq_pos rope_table rope_n_pos freq_base.
// output: "rc <status> <n>" then per backend node
//   op ne0..3 op_params[8] flags ; src: n<node index> | l<type>,<ne0>,<ne1>,<nb1>,<data>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "mi355x_ggml_mirror.hpp"

#define GGML_MAX_DIMS 4
#define GGML_MAX_SRC 10
#define GGML_MAX_OP_PARAMS 64
#define GGML_MAX_NAME 64
#define GGML_TENSOR_FLAG_OUTPUT 2

struct ggml_tensor {
    int type;
    int op;  // index into op_names below
    int64_t ne[GGML_MAX_DIMS];
    size_t nb[GGML_MAX_DIMS];
    int32_t op_params[GGML_MAX_OP_PARAMS / sizeof(int32_t)];
    int32_t flags;
    struct ggml_tensor *src[GGML_MAX_SRC];
    struct ggml_tensor *view_src;
    size_t view_offs;
    void *data;
    char name[GGML_MAX_NAME];
};

static std::vector<std::string> op_names;
static const char *ggml_op_name_of(const ggml_tensor *t) { return op_names[(size_t)t->op].c_str(); }

static int self_checks() {
    int bad = 0;
    // ops the backend does not take map to -1 (the lowering then refuses the graph)
    bad += mi355x_adapter::gop_of_name("FLASH_ATTN_EXT") != -1;
    bad += mi355x_adapter::gop_of_name("MUL_MAT") != MI355X_GOP_MUL_MAT;
    bad += mi355x_adapter::gop_of_name("CPY") != MI355X_GOP_CPY;
    const int64_t k[3] = {5, 6, 7};
    const int32_t p[3] = {5, 6, 7}, q[3] = {5, 6, 8};
    bad += !mi355x_adapter::cells_eq_pos(k, p, 3);
    bad += mi355x_adapter::cells_eq_pos(k, q, 3);  // a moved cell
    bad += mi355x_adapter::cells_eq_pos(k, p, 0);  // empty batch
    // KQ mask rows (n_kv 8): causal over [0, pos] passes; another sequence's cell inside
    // [0, pos] (-INF there), a visible cell after pos, or a wrong type is refused
    const float NI = -__builtin_inff();
    float m32[2][8];
    uint16_t m16[2][8];
    const int32_t pp[2] = {2, 5};
    for (int t = 0; t < 2; ++t)
        for (int j = 0; j < 8; ++j) {
            m32[t][j] = j <= pp[t] ? 0.f : NI;
            m16[t][j] = j <= pp[t] ? 0 : 0xfc00;
        }
    bad += !mi355x_adapter::kq_mask_causal(m32, 0, 8, 32, pp, 2);
    bad += !mi355x_adapter::kq_mask_causal(m16, 1, 8, 16, pp, 2);
    bad += mi355x_adapter::kq_mask_causal(m16, 0, 8, 16, pp, 2);
    m32[1][3] = NI;  // cell 3 belongs to another sequence
    bad += mi355x_adapter::kq_mask_causal(m32, 0, 8, 32, pp, 2);
    m32[1][3] = 0.f;
    m32[0][4] = 0.f;  // a visible cell after the position
    bad += mi355x_adapter::kq_mask_causal(m32, 0, 8, 32, pp, 2);
    m32[0][4] = NI;
    bad += !mi355x_adapter::kq_mask_causal(m32, 0, 8, 32, pp, 2);
    const int32_t far[1] = {8};  // position past the mask
    bad += mi355x_adapter::kq_mask_causal(m32, 0, 8, 32, far, 1);
    return bad;
}

int main(int argc, char **argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s graph.txt cells_eq_pos rope_table rope_n_pos freq_base\n", argv[0]);
        return 2;
    }
    if (const int bad = self_checks()) {
        std::printf("self_checks_failed %d\n", bad);
        return 1;
    }
    std::ifstream in(argv[1]);
    std::unordered_map<long, ggml_tensor *> byid;
    std::vector<std::vector<long>> refs;  // per tensor: src[10], view_src
    std::vector<ggml_tensor *> all, nodes;
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream s(line);
        std::string tag;
        s >> tag;
        if (tag == "T") {
            auto *t = new ggml_tensor();
            long id;
            std::string opn, name;
            s >> id >> t->type >> opn;
            size_t k = 0;
            while (k < op_names.size() && op_names[k] != opn) ++k;
            if (k == op_names.size()) op_names.push_back(opn);
            t->op = (int)k;
            for (auto &v : t->ne) s >> v;
            for (auto &v : t->nb) s >> v;
            for (auto &v : t->op_params) s >> v;
            s >> t->flags;
            std::vector<long> r(GGML_MAX_SRC + 1);
            for (auto &v : r) s >> v;
            unsigned long long data;
            s >> t->view_offs >> data >> name;
            t->data = (void *)(uintptr_t)data;
            if (name != "-") std::strncpy(t->name, name.c_str(), GGML_MAX_NAME - 1);
            byid[id] = t;
            all.push_back(t);
            refs.push_back(r);
        } else if (tag == "N") {
            int n;
            s >> n;
            for (int i = 0; i < n; ++i) {
                long id;
                s >> id;
                nodes.push_back(byid.at(id));
            }
        }
    }
    for (size_t i = 0; i < all.size(); ++i) {
        for (int j = 0; j < GGML_MAX_SRC; ++j) all[i]->src[j] = refs[i][j] >= 0 ? byid.at(refs[i][j]) : nullptr;
        all[i]->view_src = refs[i][GGML_MAX_SRC] >= 0 ? byid.at(refs[i][GGML_MAX_SRC]) : nullptr;
    }

    mi355x_adapter::Context ctx;
    ctx.rope_table = (void *)(uintptr_t)std::strtoull(argv[3], nullptr, 0);
    ctx.rope_n_pos = std::atoi(argv[4]);
    ctx.freq_base = (float)std::atof(argv[5]);
    mi355x_adapter::Mirror<ggml_tensor> mir;
    mir.op_name = ggml_op_name_of;
    mir.output_flag = GGML_TENSOR_FLAG_OUTPUT;
    mir.max_src = GGML_MAX_SRC;
    int nn = 0;
    const int rc = mi355x_adapter::lower(ctx, mir, nodes.data(), (int)nodes.size(), std::atoi(argv[2]) != 0, &nn);
    std::printf("rc %d %d\n", rc, rc == 0 ? nn : 0);
    if (rc) return 0;
    std::unordered_map<const mi355x_tensor *, int> idx;
    for (int i = 0; i < nn; ++i) idx[ctx.nodes[(size_t)i]] = i;
    for (int i = 0; i < nn; ++i) {
        const mi355x_tensor *t = ctx.nodes[(size_t)i];
        std::printf("%d %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64, t->op, t->ne[0], t->ne[1], t->ne[2], t->ne[3]);
        for (int p = 0; p < 8; ++p) std::printf(" %d", t->op_params[p]);
        std::printf(" %d ;", t->flags);
        for (int s = 0; s < MI355X_MAX_SRC && t->src[s]; ++s) {
            const mi355x_tensor *u = t->src[s];
            auto it = idx.find(u);
            if (it != idx.end())
                std::printf(" n%d", it->second);
            else
                std::printf(" l%d,%" PRId64 ",%" PRId64 ",%zu,%" PRIuPTR, u->type, u->ne[0], u->ne[1], u->nb[1],
                            (uintptr_t)u->data);
        }
        std::printf("\n");
    }
    for (auto *t : all) delete t;
    return 0;
}
