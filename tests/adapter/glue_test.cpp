// glue_test.cpp — drives the ggml-backend registration (adapter/ggml-mi355x.cpp) the way
// llama.cpp's backend registry and scheduler do: reg -> device -> props / supports_op ->
// init_backend -> buffer type -> alloc_buffer -> set_tensor -> graph_compute -> get_tensor.
// Test infrastructure (tests/test_adapter.py, tests/test_gpu_adapter.py), compiled with
// -Werror against the restated ggml headers in tests/adapter/ggml/ and the stub of the
// ggml calls the glue makes (ggml_stub.cpp).
//
//   glue_test reg
//       registry / DL entry checks; prints "devices <n>" (0 on a host without a GPU).
//   glue_test decode graph.txt blob.bin tokens.txt out.bin buffer_bytes n_vocab
//       graph.txt: tensors as tests/test_adapter.py serializes them, data = BASE + offset
//       for tensors in the backend buffer (BASE = 1 << 44); blob.bin: [u64 off][u64 n][n
//       bytes]... uploaded with set_tensor; tokens.txt: token ids, one per position. Per
//       token: the graph inputs (inp_tokens, inp_pos, k_idxs, v_idxs, the f16 / f32 KQ
//       mask causal over [0, pos]) set through the buffer (even positions) or the
//       backend's async set (odd), graph_compute, the logits (the last node) read back into
//       out.bin. Then a mask that hides cell 0 at the next position must be refused.
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "ggml-backend-impl.h"
#include "ggml-mi355x.h"
#include "ggml_mi355x.h"
#include "ggml_stub.h"

extern "C" ggml_backend_reg_t ggml_backend_init(void);
extern "C" int ggml_backend_score(void);

static const uint64_t BASE = 1ull << 44;

#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);         \
            return 1;                                                       \
        }                                                                   \
    } while (0)

static int reg_checks(int *n_out) {
    ggml_backend_reg_t reg = ggml_backend_mi355x_reg();
    CHECK(reg && reg->api_version == GGML_BACKEND_API_VERSION);
    CHECK(std::strcmp(reg->iface.get_name(reg), "MI355X") == 0);
    CHECK(ggml_backend_init() == reg);  // GGML_BACKEND_DL_IMPL
    const size_t n = reg->iface.get_device_count(reg);
    CHECK((int)n == mi355x_device_count() && (int)n == ggml_backend_mi355x_get_device_count());
    CHECK(ggml_backend_score() == (n ? 10 : 0));
    CHECK(reg->iface.get_device(reg, n) == nullptr);
    CHECK(ggml_backend_mi355x_init((int)n) == nullptr);
    CHECK(ggml_backend_mi355x_buffer_type(-1) == nullptr);
    CHECK(reg->iface.get_proc_address(reg, "ggml_backend_set_n_threads") == nullptr);
    for (size_t i = 0; i < n; ++i) {
        ggml_backend_dev_t dev = reg->iface.get_device(reg, i);
        CHECK(dev && dev->reg == reg);
        ggml_backend_dev_props p;
        dev->iface.get_props(dev, &p);
        CHECK(p.type == GGML_BACKEND_DEVICE_TYPE_GPU && p.memory_total > 0 && p.memory_free <= p.memory_total);
        CHECK(std::strncmp(p.name, "MI355X", 6) == 0);
        ggml_backend_buffer_type_t buft = dev->iface.get_buffer_type(dev);
        CHECK(buft == ggml_backend_mi355x_buffer_type((int)i) && buft->device == dev);
        CHECK(dev->iface.supports_buft(dev, buft) && !buft->iface.is_host(buft));
        CHECK(buft->iface.get_alignment(buft) == 256);
        ggml_backend_t be = ggml_backend_mi355x_init((int)i);
        CHECK(be && ggml_backend_is_mi355x(be) && be->device == dev);
        be->iface.free(be);
    }
    *n_out = (int)n;
    return 0;
}

// supports_op on hand-made nodes: what the scheduler asks before placing a node
static int supports_checks(ggml_backend_dev_t dev) {
    ggml_tensor w{}, x{}, y{}, ids{}, g{}, u{}, s{};
    auto shape = [](ggml_tensor &t, ggml_type ty, int64_t ne0, int64_t ne1, size_t nb0, size_t nb1) {
        t.type = ty;
        t.ne[0] = ne0, t.ne[1] = ne1, t.ne[2] = t.ne[3] = 1;
        t.nb[0] = nb0, t.nb[1] = nb1, t.nb[2] = t.nb[3] = nb1 * (size_t)ne1;
    };
    shape(w, GGML_TYPE_Q4_K, 2048, 512, 144, 8 * 144);
    shape(x, GGML_TYPE_F32, 2048, 1, 4, 2048 * 4);
    shape(y, GGML_TYPE_F32, 512, 1, 4, 512 * 4);
    y.op = GGML_OP_MUL_MAT;
    y.src[0] = &w, y.src[1] = &x;
    CHECK(dev->iface.supports_op(dev, &y));
    CHECK(!dev->iface.offload_op(dev, &y));  // decode: stays where the weights are
    x.ne[1] = y.ne[1] = 64;
    x.nb[2] = x.nb[3] = x.nb[1] * 64;
    y.nb[2] = y.nb[3] = y.nb[1] * 64;
    CHECK(dev->iface.supports_op(dev, &y) && dev->iface.offload_op(dev, &y));  // prompt batch
    w.type = GGML_TYPE_Q8_0;  // not a K-quant
    CHECK(!dev->iface.supports_op(dev, &y));
    w.type = GGML_TYPE_Q6_K;
    w.nb[0] = 210, w.nb[1] = 8 * 210;
    CHECK(dev->iface.supports_op(dev, &y));
    w.ne[0] = 1024;  // K mismatch
    CHECK(!dev->iface.supports_op(dev, &y));
    shape(g, GGML_TYPE_F32, 5632, 1, 4, 5632 * 4);
    shape(u, GGML_TYPE_F32, 5632, 1, 4, 5632 * 4);
    shape(s, GGML_TYPE_F32, 5632, 1, 4, 5632 * 4);
    s.op = GGML_OP_GLU;
    s.src[0] = &g, s.src[1] = &u;
    s.op_params[0] = GGML_GLU_OP_SWIGLU;
    CHECK(dev->iface.supports_op(dev, &s));
    s.op_params[0] = GGML_GLU_OP_GEGLU;
    CHECK(!dev->iface.supports_op(dev, &s));
    s.op = GGML_OP_FLASH_ATTN_EXT;
    CHECK(!dev->iface.supports_op(dev, &s));
    s.op = GGML_OP_UNARY;
    CHECK(!dev->iface.supports_op(dev, &s));
    shape(ids, GGML_TYPE_I32, 1, 1, 4, 4);
    shape(w, GGML_TYPE_Q4_K, 2048, 32000, 144, 8 * 144);
    shape(y, GGML_TYPE_F32, 2048, 1, 4, 2048 * 4);
    y.op = GGML_OP_GET_ROWS;
    y.src[0] = &w, y.src[1] = &ids;
    CHECK(dev->iface.supports_op(dev, &y));
    // f16 MUL_MAT: only the attention's KQ / KQV on a view of the f16 KV cache is claimed;
    // an F16 lm_head (or tied embedding) stays on the CPU backend
    ggml_tensor hw{}, hx{}, hy{}, kc{}, kv{}, rq{}, rp{}, kq{}, ct{};
    shape(hw, GGML_TYPE_F16, 2048, 32000, 2, 2048 * 2);
    shape(hx, GGML_TYPE_F32, 2048, 1, 4, 2048 * 4);
    shape(hy, GGML_TYPE_F32, 32000, 1, 4, 32000 * 4);
    hy.op = GGML_OP_MUL_MAT;
    hy.src[0] = &hw, hy.src[1] = &hx;
    CHECK(!dev->iface.supports_op(dev, &hy));
    shape(kc, GGML_TYPE_F16, 256, 128, 2, 256 * 2);  // K cache leaf [n_ctx][n_head_kv * hd]
    shape(kv, GGML_TYPE_F16, 64, 128, 2, 256 * 2);   // one kv head's view from cell 0
    kv.op = GGML_OP_VIEW;
    kv.src[0] = &kc, kv.view_src = &kc;
    shape(rq, GGML_TYPE_F32, 64, 32, 4, 64 * 4);
    rq.op = GGML_OP_ROPE;
    shape(rp, GGML_TYPE_F32, 64, 1, 4, 64 * 4);
    rp.op = GGML_OP_PERMUTE;
    rp.src[0] = &rq;
    shape(kq, GGML_TYPE_F32, 128, 1, 4, 128 * 4);
    kq.op = GGML_OP_MUL_MAT;
    kq.src[0] = &kv, kq.src[1] = &rp;
    CHECK(dev->iface.supports_op(dev, &kq));
    kq.src[1] = &hx;  // the same view against a plain activation: not the attention pattern
    CHECK(!dev->iface.supports_op(dev, &kq));
    kv.view_offs = 512;  // a view that does not start at cell 0
    kq.src[1] = &rp;
    CHECK(!dev->iface.supports_op(dev, &kq));
    // CONT / CPY: only CONT(PERMUTE(KQV)) is lowered
    shape(ct, GGML_TYPE_F32, 64, 1, 4, 64 * 4);
    ct.op = GGML_OP_CONT;
    ct.src[0] = &rp;  // PERMUTE(ROPE): not an attention output
    CHECK(!dev->iface.supports_op(dev, &ct));
    ct.op = GGML_OP_CPY;
    ct.src[0] = &hx;
    CHECK(!dev->iface.supports_op(dev, &ct));
    return 0;
}

struct Loaded {
    std::vector<ggml_tensor *> all, nodes;
    std::unordered_map<std::string, ggml_tensor *> by_name;
};

static bool load_graph(const char *path, Loaded &L, char *base) {
    std::ifstream in(path);
    std::unordered_map<long, ggml_tensor *> byid;
    std::vector<std::vector<long>> refs;
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream s(line);
        std::string tag;
        s >> tag;
        if (tag == "T") {
            auto *t = new ggml_tensor();
            long id;
            int type;
            std::string opn, name;
            s >> id >> type >> opn;
            t->type = (ggml_type)type;
            t->op = stub_op_of_name(opn.c_str());
            if (t->op == GGML_OP_COUNT) return false;
            for (auto &v : t->ne) s >> v;
            for (auto &v : t->nb) s >> v;
            for (auto &v : t->op_params) s >> v;
            s >> t->flags;
            std::vector<long> r(GGML_MAX_SRC + 1);
            for (auto &v : r) s >> v;
            unsigned long long data;
            s >> t->view_offs >> data >> name;
            t->data = data >= BASE ? (void *)(base + (data - BASE)) : (void *)(uintptr_t)data;
            if (name != "-") std::strncpy(t->name, name.c_str(), GGML_MAX_NAME - 1);
            if (!L.by_name.count(t->name)) L.by_name[t->name] = t;
            byid[id] = t;
            L.all.push_back(t);
            refs.push_back(r);
        } else if (tag == "N") {
            int n;
            s >> n;
            for (int i = 0; i < n; ++i) {
                long id;
                s >> id;
                L.nodes.push_back(byid.at(id));
            }
        }
    }
    for (size_t i = 0; i < L.all.size(); ++i) {
        for (int j = 0; j < GGML_MAX_SRC; ++j) L.all[i]->src[j] = refs[i][j] >= 0 ? byid.at(refs[i][j]) : nullptr;
        L.all[i]->view_src = refs[i][GGML_MAX_SRC] >= 0 ? byid.at(refs[i][GGML_MAX_SRC]) : nullptr;
    }
    return !L.nodes.empty();
}

static void set_input(ggml_backend_t be, ggml_backend_buffer_t buf, ggml_tensor *t, const void *data, size_t n,
                      bool async) {
    if (async) {
        be->iface.set_tensor_async(be, t, data, 0, n);
        be->iface.synchronize(be);
    } else {
        buf->iface.set_tensor(buf, t, data, 0, n);
    }
}

static int decode(int argc, char **argv) {
    if (argc < 8) return 2;
    const size_t buf_bytes = std::strtoull(argv[6], nullptr, 0);
    const int64_t n_vocab = std::atoll(argv[7]);
    ggml_backend_reg_t reg = ggml_backend_mi355x_reg();
    CHECK(reg->iface.get_device_count(reg) >= 1);
    ggml_backend_dev_t dev = reg->iface.get_device(reg, 0);
    if (supports_checks(dev)) return 1;
    ggml_backend_t be = dev->iface.init_backend(dev, nullptr);
    CHECK(be != nullptr);
    ggml_backend_buffer_type_t buft = dev->iface.get_buffer_type(dev);
    ggml_backend_buffer_t buf = buft->iface.alloc_buffer(buft, buf_bytes);
    CHECK(buf && buf->size == buf_bytes && buf->buft == buft);
    char *base = (char *)buf->iface.get_base(buf);
    buf->iface.clear(buf, 0);

    Loaded L;
    CHECK(load_graph(argv[2], L, base));
    for (ggml_tensor *t : L.all) {
        if ((char *)t->data >= base && (char *)t->data < base + buf_bytes) {
            t->buffer = buf;
            CHECK(buf->iface.init_tensor(buf, t) == GGML_STATUS_SUCCESS);
        }
    }
    // weights and norms: one set_tensor per blob record (the bytes unchanged)
    {
        std::ifstream bin(argv[3], std::ios::binary);
        ggml_tensor whole{};
        whole.data = base;
        whole.buffer = buf;
        uint64_t hdr[2];
        std::vector<char> bytes;
        int records = 0;
        while (bin.read((char *)hdr, sizeof(hdr))) {
            bytes.resize(hdr[1]);
            bin.read(bytes.data(), (std::streamsize)hdr[1]);
            CHECK(hdr[0] + hdr[1] <= buf_bytes);
            buf->iface.set_tensor(buf, &whole, bytes.data(), hdr[0], hdr[1]);
            ++records;
        }
        std::printf("uploaded %d\n", records);
    }
    int unsupported = 0;
    for (ggml_tensor *t : L.nodes) unsupported += !dev->iface.supports_op(dev, t);
    std::printf("unsupported %d\n", unsupported);

    ggml_tensor *tok = L.by_name.at("inp_tokens"), *pos = L.by_name.at("inp_pos"), *mask = L.by_name.at("kq_mask");
    ggml_tensor *kid = L.by_name.at("k_idxs"), *vid = L.by_name.at("v_idxs");
    ggml_tensor *logits = L.nodes.back();
    CHECK(logits->ne[0] == n_vocab && (logits->flags & GGML_TENSOR_FLAG_OUTPUT));
    const int64_t n_kv = mask->ne[0];
    ggml_cgraph *cg = stub_graph_new(L.nodes.data(), (int)L.nodes.size());
    std::vector<int32_t> tokens;
    {
        std::ifstream tin(argv[4]);
        int32_t v;
        while (tin >> v) tokens.push_back(v);
    }
    auto set_inputs = [&](int p, int32_t token, bool async, int hide_cell) {
        const int32_t tp[1] = {token}, pp[1] = {p};
        set_input(be, buf, tok, tp, 4, async);
        set_input(be, buf, pos, pp, 4, async);
        const int64_t kk[1] = {p};
        set_input(be, buf, kid, kk, 8, async);
        std::vector<int64_t> vv((size_t)ggml_nelements(vid));
        for (size_t i = 0; i < vv.size(); ++i) vv[i] = (int64_t)i * n_kv + p;
        set_input(be, buf, vid, vv.data(), vv.size() * 8, async);
        std::vector<uint8_t> m((size_t)mask->nb[1]);
        for (int64_t j = 0; j < n_kv; ++j) {
            const bool vis = j <= p && j != hide_cell;
            if (mask->type == GGML_TYPE_F16) {
                const uint16_t h = vis ? 0 : 0xfc00;
                std::memcpy(m.data() + 2 * j, &h, 2);
            } else {
                const float f = vis ? 0.f : -INFINITY;
                std::memcpy(m.data() + 4 * j, &f, 4);
            }
        }
        set_input(be, buf, mask, m.data(), m.size(), async);
    };
    FILE *out = std::fopen(argv[5], "wb");
    CHECK(out != nullptr);
    std::vector<float> lg((size_t)n_vocab);
    for (size_t p = 0; p < tokens.size(); ++p) {
        set_inputs((int)p, tokens[p], (p & 1) != 0, -1);
        const ggml_status st = be->iface.graph_compute(be, cg);
        be->iface.synchronize(be);
        std::printf("token %zu status %d\n", p, (int)st);
        CHECK(st == GGML_STATUS_SUCCESS);
        buf->iface.get_tensor(buf, logits, lg.data(), 0, lg.size() * 4);
        std::fwrite(lg.data(), 4, lg.size(), out);
    }
    std::fclose(out);
    // another sequence's cell (or a removed one) inside [0, pos]: the promise does not hold,
    // the attention block is not lowered, the graph is refused -- never computed wrongly
    const int p = (int)tokens.size();
    set_inputs(p, tokens.back(), false, 0);
    const ggml_status st = be->iface.graph_compute(be, cg);
    be->iface.synchronize(be);
    std::printf("refused %d\n", (int)st);
    CHECK(st == GGML_STATUS_FAILED);
    stub_graph_free(cg);
    buf->iface.free_buffer(buf);
    delete buf;
    be->iface.free(be);
    for (ggml_tensor *t : L.all) delete t;
    std::printf("ok\n");
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    if (std::strcmp(argv[1], "reg") == 0) {
        int n = 0;
        if (reg_checks(&n)) return 1;
        if (n > 0 && supports_checks(ggml_backend_mi355x_reg()->iface.get_device(ggml_backend_mi355x_reg(), 0)))
            return 1;
        std::printf("devices %d\nok\n", n);
        return 0;
    }
    if (std::strcmp(argv[1], "decode") == 0) return decode(argc, argv);
    return 2;
}
