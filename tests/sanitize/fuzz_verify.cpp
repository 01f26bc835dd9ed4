// Mutation driver for the untrusted-input path of libxfgstark (proof parser + host verifier),
// built host-only with AddressSanitizer + UndefinedBehaviorSanitizer (xfg-stark_amd/Makefile
// target `sanitize`; run by tests/test_sanitize.py on the CPU).
//
// Reference side of this path: XfgBurnMintVerifier::verify_with_public_inputs ->
// winterfell::verify (src/burn_mint_verifier.rs:186-283), which deserialises attacker-supplied
// proof bytes. Every mutated proof must be REJECTED (never accepted, never a crash, leak or UB):
//   * truncation at every length 0 .. len-1 (every section boundary included),
//   * every byte set to 0x00, 0xFF, xor 0x80 and +1 (u8 counts out of range, inflated u16/u32
//     length fields, flipped digests / elements / nonce),
//   * at every offset (step `stride`), 8 bytes overwritten with p, p + 1 and 2^64 - 1 (field
//     elements >= p),
//   * the untouched proof appended with trailing bytes.
// The untouched proof must be accepted. Exit status 0 = all as expected; the counts go to stdout.
//
// usage: fuzz_verify <proof file> <air file: 14 LE u64> q beta grinding ext fold remdeg [stride]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/xfg_stark.h"

static std::vector<uint8_t> slurp(const char* path) {
    std::vector<uint8_t> v;
    FILE* f = fopen(path, "rb");
    if (!f) return v;
    uint8_t buf[65536];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + k);
    fclose(f);
    return v;
}

struct Ctx {
    xfg_air_consts air;
    xfg_options opt;
    long accepted_bad = 0, checked = 0;
    // parse + verify one candidate on an exactly-sized heap copy (ASan sees any overread)
    int run(const uint8_t* p, size_t len, bool expect_ok) {
        uint8_t* b = (uint8_t*)malloc(len ? len : 1);
        if (len) memcpy(b, p, len);
        xfg_proof_info info;
        char err[256];
        const int ps = xfg_proof_parse(b, len, &info, err, sizeof err);
        const int vs = xfg_verify(b, len, &air, &opt, err, sizeof err);
        free(b);
        checked++;
        if (ps != XFG_OK && vs == XFG_OK) {
            fprintf(stderr, "verify accepted a proof the parser rejected (len %zu)\n", len);
            accepted_bad++;
        }
        if (!expect_ok && vs == XFG_OK) accepted_bad++;
        if (expect_ok && vs != XFG_OK) {
            fprintf(stderr, "untouched proof rejected: %s\n", err);
            return 1;
        }
        return 0;
    }
};

int main(int argc, char** argv) {
    if (argc < 9) {
        fprintf(stderr, "usage: %s proof air q beta grinding ext fold remdeg [stride]\n", argv[0]);
        return 2;
    }
    std::vector<uint8_t> proof = slurp(argv[1]), airb = slurp(argv[2]);
    if (proof.empty() || airb.size() != 14 * 8) {
        fprintf(stderr, "bad inputs\n");
        return 2;
    }
    Ctx c;
    memcpy(c.air.pub_inputs, airb.data(), 12 * 8);
    memcpy(&c.air.nullifier, airb.data() + 96, 8);
    memcpy(&c.air.commitment, airb.data() + 104, 8);
    c.opt = {(uint32_t)atoi(argv[3]), (uint32_t)atoi(argv[4]), (uint32_t)atoi(argv[5]), (uint32_t)atoi(argv[6]),
             (uint32_t)atoi(argv[7]), (uint32_t)atoi(argv[8])};
    const size_t stride = argc > 9 ? (size_t)atoi(argv[9]) : 1;
    const size_t L = proof.size();
    if (c.run(proof.data(), L, true)) return 1;

    for (size_t k = 0; k < L; k++) c.run(proof.data(), k, false);  // truncations
    std::vector<uint8_t> m(proof);
    for (size_t i = 0; i < L; i += stride) {  // byte mutations
        const uint8_t o = m[i];
        const uint8_t vals[4] = {0x00, 0xFF, (uint8_t)(o ^ 0x80), (uint8_t)(o + 1)};
        for (uint8_t v : vals) {
            if (v == o) continue;
            m[i] = v;
            c.run(m.data(), L, false);
        }
        m[i] = o;
    }
    const uint64_t P = 0xFFFFFFFF00000001ULL;
    const uint64_t big[3] = {P, P + 1, ~0ULL};
    for (size_t i = 0; i + 8 <= L; i += stride) {  // non-canonical elements anywhere
        uint8_t save[8];
        memcpy(save, &m[i], 8);
        for (uint64_t v : big) {
            if (!memcmp(&v, save, 8)) continue;
            memcpy(&m[i], &v, 8);
            c.run(m.data(), L, false);
        }
        memcpy(&m[i], save, 8);
    }
    std::vector<uint8_t> tail(proof);  // trailing bytes
    tail.push_back(0);
    c.run(tail.data(), tail.size(), false);

    // the batch entry point over a mix of good and mutated proofs (host threads)
    std::vector<std::vector<uint8_t>> items = {proof, std::vector<uint8_t>(proof.begin(), proof.begin() + L / 2), tail};
    std::vector<const uint8_t*> ptrs;
    std::vector<size_t> lens;
    std::vector<xfg_air_consts> airs(items.size(), c.air);
    for (auto& it : items) {
        ptrs.push_back(it.data());
        lens.push_back(it.size());
    }
    std::vector<int> res(items.size(), -1);
    if (xfg_verify_batch((uint32_t)items.size(), ptrs.data(), lens.data(), airs.data(), &c.opt, res.data(), 3) != XFG_OK ||
        res[0] != XFG_OK || res[1] == XFG_OK || res[2] == XFG_OK) {
        fprintf(stderr, "batch verify verdicts wrong: %d %d %d\n", res[0], res[1], res[2]);
        return 1;
    }
    printf("checked %ld mutated proofs of %zu bytes, accepted %ld\n", c.checked, L, c.accepted_bad);
    return c.accepted_bad ? 1 : 0;
}
