// flopcount.cpp — algorithmic FLOP count of one per-point DAE evaluation
// (TEST / MEASUREMENT INFRASTRUCTURE; SURVEY.md §8(d): "F_dae counted
// exactly by running the CPU restatement with a flop-counting scalar type").
// Compiles oracle.c as C++ with `real` = Counted; every +,-,*,/ on model
// values counts 1, every elementary function (sqrt, exp, log, sin, cos,
// tanh, sinh, pow) counts 1 and is tallied separately.
#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>

#include "../include/mocohip.h"

struct FlopTally {
    double add = 0, mul = 0, div = 0, fn = 0;
};
static FlopTally g_tally;

struct Counted {
    double v;
    Counted() = default;
    Counted(double x) : v(x) {}
    Counted(int x) : v(x) {}
    Counted& operator+=(const Counted& o) { g_tally.add++; v += o.v; return *this; }
    Counted& operator-=(const Counted& o) { g_tally.add++; v -= o.v; return *this; }
    Counted& operator*=(const Counted& o) { g_tally.mul++; v *= o.v; return *this; }
    Counted& operator/=(const Counted& o) { g_tally.div++; v /= o.v; return *this; }
};
static inline Counted operator+(Counted a, Counted b) { g_tally.add++; return Counted(a.v + b.v); }
static inline Counted operator-(Counted a, Counted b) { g_tally.add++; return Counted(a.v - b.v); }
static inline Counted operator*(Counted a, Counted b) { g_tally.mul++; return Counted(a.v * b.v); }
static inline Counted operator/(Counted a, Counted b) { g_tally.div++; return Counted(a.v / b.v); }
static inline Counted operator-(Counted a) { return Counted(-a.v); }
static inline bool operator<(Counted a, Counted b) { return a.v < b.v; }
static inline bool operator>(Counted a, Counted b) { return a.v > b.v; }
static inline bool operator<=(Counted a, Counted b) { return a.v <= b.v; }
static inline bool operator>=(Counted a, Counted b) { return a.v >= b.v; }
static inline bool operator==(Counted a, Counted b) { return a.v == b.v; }
#define CFN(name) \
    static inline Counted name(Counted a) { g_tally.fn++; return Counted(std::name(a.v)); }
CFN(sqrt) CFN(exp) CFN(log) CFN(sin) CFN(cos) CFN(tanh) CFN(sinh) CFN(asin) CFN(acos)
static inline Counted atan2(Counted a, Counted b) { g_tally.fn++; return Counted(std::atan2(a.v, b.v)); }
static inline Counted fabs(Counted a) { return Counted(std::fabs(a.v)); }
static inline Counted pow(Counted a, double b) { g_tally.fn++; return Counted(std::pow(a.v, b)); }
static inline bool isnan(Counted a) { return std::isnan(a.v); }

#define ORACLE_REAL Counted
#define ORACLE_COUNTING 1
#include "oracle.c"

extern "C" {
// Evaluate the DAE once at `input` = [time, states, controls] and return the
// tallies [add/sub, mul, div, elementary functions].
int orc_count_dae_flops(const mh_problem* p, const mh_options* o, const double* input,
        double* tally4, double* outputs) {
    orc_ctx* c = nullptr;
    int rc = orc_create(p, o, &c);
    if (rc) return rc;
    dae_ws w;
    ws_alloc(c, &w);
    int NI = c->NS + c->NC, NO = c->NQ + c->NZ;
    Counted* in = new Counted[NI + 1];
    Counted* out = new Counted[NO + 1];
    for (int i = 0; i < NI; ++i) in[i] = Counted(input[1 + i]);
    g_tally = FlopTally();
    eval_dae_point(c, &w, Counted(input[0]), in, in + c->NS, out);
    tally4[0] = g_tally.add;
    tally4[1] = g_tally.mul;
    tally4[2] = g_tally.div;
    tally4[3] = g_tally.fn;
    for (int i = 0; i < NO; ++i) outputs[i] = out[i].v;
    delete[] in;
    delete[] out;
    ws_free(&w);
    orc_destroy(c);
    return 0;
}
}
