// lgs_posegraph.cpp -- PoseGraph, robust losses and PoseGraphOptimizerLM
// (see lgs_posegraph.hpp for the reference map).
#include "lgs_posegraph.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <queue>
#include <stdexcept>
#include <unordered_map>

namespace MyLidarGraphSlam {
namespace Hip {
namespace Mapping {

using Mat3 = std::array<double, 9>;   // row-major
using Vec3 = std::array<double, 3>;

// ---------------------------------------------------------------------------
// pose algebra (H/pose.hpp:150-206, H/util.hpp:125-135)
// ---------------------------------------------------------------------------
RobotPose2D<double> InverseCompound(const RobotPose2D<double>& s, const RobotPose2D<double>& e)
{
    double sinT, cosT;
    sincos(s.mTheta, &sinT, &cosT);
    const double dx = e.mX - s.mX, dy = e.mY - s.mY, dt = e.mTheta - s.mTheta;
    return RobotPose2D<double>(cosT * dx + sinT * dy, -sinT * dx + cosT * dy, dt);
}

RobotPose2D<double> Compound(const RobotPose2D<double>& s, const RobotPose2D<double>& d)
{
    double sinT, cosT;
    sincos(s.mTheta, &sinT, &cosT);
    return RobotPose2D<double>(s.mX + cosT * d.mX - sinT * d.mY, s.mY + sinT * d.mX + cosT * d.mY,
                               s.mTheta + d.mTheta);
}

double NormalizeAngle(double theta)
{
    double t = std::fmod(theta, 2.0 * M_PI);
    if (t > M_PI)
        t -= 2.0 * M_PI;
    else if (t < -M_PI)
        t += 2.0 * M_PI;
    return t;
}

// ---------------------------------------------------------------------------
// PoseGraph (C/mapping/pose_graph.cpp)
// ---------------------------------------------------------------------------
int PoseGraph::AppendNode(const RobotPose2D<double>& pose, double timeStamp)
{
    const int idx = static_cast<int>(mNodes.size());
    mNodes.emplace_back(idx, pose, timeStamp);
    return idx;
}

void PoseGraph::AppendEdge(int startNodeIdx, int endNodeIdx, const RobotPose2D<double>& relativePose,
                           const Matrix3d& informationMat)
{
    mEdges.emplace_back(startNodeIdx, endNodeIdx, relativePose, informationMat);
}

// ---------------------------------------------------------------------------
// robust losses (C/mapping/robust_loss_function.cpp), same expressions
// ---------------------------------------------------------------------------
double LossHuber::Loss(double t) const { return (t <= mScale) ? t : (2.0 * std::sqrt(mScale * t) - mScale); }
double LossHuber::Weight(double t) const { return (t <= mScale) ? 1.0 : std::sqrt(mScale / t); }
double LossCauchy::Loss(double t) const { return mScale * std::log1p(t / mScale); }
double LossCauchy::Weight(double t) const { return mScale / (mScale + t); }
double LossFair::Loss(double t) const
{
    const double e = std::sqrt(t / mScale);
    return 2.0 * mScale * (e - std::log1p(e));
}
double LossFair::Weight(double t) const
{
    const double e = std::sqrt(t / mScale);
    return 1.0 / (1.0 + e);
}
double LossGemanMcClure::Loss(double t) const { return mScale * t / (mScale + t); }
double LossGemanMcClure::Weight(double t) const
{
    const double s2 = mScale * mScale, st = mScale + t;
    return s2 / (st * st);
}
double LossWelsch::Loss(double t) const { return mScale * (-std::expm1(-t / mScale)); }
double LossWelsch::Weight(double t) const { return std::exp(-t / mScale); }
double LossDCS::Loss(double t) const { return mScale * t / (mScale + t); }
double LossDCS::Weight(double t) const
{
    return (t <= mScale) ? 1.0 : std::pow(2.0 * mScale / (t + mScale), 2.0);
}

LossFunctionPtr CreateLossFunction(int kind, double scale)
{
    switch (kind) {
    case 0: return std::make_shared<LossHuber>(scale);
    case 1: return std::make_shared<LossCauchy>(scale);
    case 2: return std::make_shared<LossFair>(scale);
    case 3: return std::make_shared<LossGemanMcClure>(scale);
    case 4: return std::make_shared<LossWelsch>(scale);
    case 5: return std::make_shared<LossDCS>(scale);
    case 6: return std::make_shared<LossSquared>();
    default: return nullptr;
    }
}

// ---------------------------------------------------------------------------
// small dense helpers (each coefficient a k = 0..2 sequential sum, like a
// fixed-size Eigen product)
// ---------------------------------------------------------------------------
namespace {

inline Mat3 mul(const Mat3& a, const Mat3& b)
{
    Mat3 c;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            c[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
    return c;
}

inline Mat3 mul_tn(const Mat3& a, const Mat3& b)   // a^T b
{
    Mat3 c;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            c[3 * i + j] = a[i] * b[j] + a[3 + i] * b[3 + j] + a[6 + i] * b[6 + j];
    return c;
}

inline Mat3 mul_nt(const Mat3& a, const Mat3& b)   // a b^T
{
    Mat3 c;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            c[3 * i + j] = a[3 * i] * b[3 * j] + a[3 * i + 1] * b[3 * j + 1] + a[3 * i + 2] * b[3 * j + 2];
    return c;
}

inline Vec3 mulv(const Mat3& a, const Vec3& x)
{
    return Vec3{ a[0] * x[0] + a[1] * x[1] + a[2] * x[2], a[3] * x[0] + a[4] * x[1] + a[5] * x[2],
                 a[6] * x[0] + a[7] * x[1] + a[8] * x[2] };
}

inline Vec3 mulv_t(const Mat3& a, const Vec3& x)   // a^T x
{
    return Vec3{ a[0] * x[0] + a[3] * x[1] + a[6] * x[2], a[1] * x[0] + a[4] * x[1] + a[7] * x[2],
                 a[2] * x[0] + a[5] * x[1] + a[8] * x[2] };
}

inline Mat3 transpose(const Mat3& a) { return Mat3{ a[0], a[3], a[6], a[1], a[4], a[7], a[2], a[5], a[8] }; }

inline void sub_into(Mat3& a, const Mat3& b)
{
    for (int k = 0; k < 9; ++k) a[k] -= b[k];
}

// Lower Cholesky factor of a 3x3 SPD block
Mat3 chol3(const Mat3& a)
{
    Mat3 l{};
    l[0] = std::sqrt(a[0]);
    l[3] = a[3] / l[0];
    l[6] = a[6] / l[0];
    l[4] = std::sqrt(a[4] - l[3] * l[3]);
    l[7] = (a[7] - l[6] * l[3]) / l[4];
    l[8] = std::sqrt(a[8] - l[6] * l[6] - l[7] * l[7]);
    if (!(l[0] > 0.0 && l[4] > 0.0 && l[8] > 0.0))
        throw std::runtime_error("PoseGraphOptimizerLM: the normal matrix is not positive definite");
    return l;
}

inline Vec3 lsolve(const Mat3& l, const Vec3& b)   // L y = b
{
    Vec3 y;
    y[0] = b[0] / l[0];
    y[1] = (b[1] - l[3] * y[0]) / l[4];
    y[2] = (b[2] - l[6] * y[0] - l[7] * y[1]) / l[8];
    return y;
}

inline Vec3 ltsolve(const Mat3& l, const Vec3& b)  // L^T x = b
{
    Vec3 x;
    x[2] = b[2] / l[8];
    x[1] = (b[1] - l[7] * x[2]) / l[4];
    x[0] = (b[0] - l[3] * x[1] - l[6] * x[2]) / l[0];
    return x;
}

// B L^{-T} for the 3x3 lower factor L: each row r of B solves L x = r
inline Mat3 right_solve_lt(const Mat3& b, const Mat3& l)
{
    Mat3 c;
    for (int i = 0; i < 3; ++i) {
        const Vec3 r = lsolve(l, Vec3{ b[3 * i], b[3 * i + 1], b[3 * i + 2] });
        c[3 * i] = r[0], c[3 * i + 1] = r[1], c[3 * i + 2] = r[2];
    }
    return c;
}

// H of the normal equations in 3x3 blocks: one diagonal block per node, one
// off-diagonal block per connected node pair, stored as the block at (row a,
// column b) for a < b (the (b, a) block is its transpose).
struct BlockMatrix {
    int n = 0;
    std::vector<Mat3> diag;
    std::vector<std::pair<int, int>> pairs;     // (a, b), a < b
    std::vector<Mat3> off;                      // block (a, b)
    std::unordered_map<long long, int> index;   // a * n + b -> pair slot

    void reset(int nodes)
    {
        n = nodes;
        diag.assign(n, Mat3{});
        for (auto& m : off) m = Mat3{};
    }
    // the block at (row r, column c), r != c: accumulate x (as that block)
    void add_off(int r, int c, const Mat3& x)
    {
        const bool swap = r > c;
        const int a = swap ? c : r, b = swap ? r : c;
        const long long key = (long long)a * n + b;
        auto it = index.find(key);
        int slot;
        if (it == index.end()) {
            slot = (int)pairs.size();
            index.emplace(key, slot);
            pairs.emplace_back(a, b);
            off.push_back(Mat3{});
        } else {
            slot = it->second;
        }
        Mat3& m = off[slot];
        if (swap)
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) m[3 * j + i] += x[3 * i + j];
        else
            for (int k = 0; k < 9; ++k) m[k] += x[k];
    }
    std::vector<double> apply(const std::vector<double>& x) const
    {
        std::vector<double> y((size_t)3 * n, 0.0);
        for (int v = 0; v < n; ++v) {
            const Vec3 r = mulv(diag[v], Vec3{ x[3 * v], x[3 * v + 1], x[3 * v + 2] });
            for (int k = 0; k < 3; ++k) y[3 * v + k] += r[k];
        }
        for (size_t p = 0; p < pairs.size(); ++p) {
            const int a = pairs[p].first, b = pairs[p].second;
            const Vec3 ra = mulv(off[p], Vec3{ x[3 * b], x[3 * b + 1], x[3 * b + 2] });
            const Vec3 rb = mulv_t(off[p], Vec3{ x[3 * a], x[3 * a + 1], x[3 * a + 2] });
            for (int k = 0; k < 3; ++k) {
                y[3 * a + k] += ra[k];
                y[3 * b + k] += rb[k];
            }
        }
        return y;
    }
};

// Minimum-degree elimination order of the node graph and the fill pattern:
// order[k] = the k-th node eliminated, later[v] = the nodes adjacent to v in
// the elimination graph when v is eliminated (all eliminated after v), sorted.
void minimum_degree(const BlockMatrix& H, std::vector<int>& order, std::vector<std::vector<int>>& later)
{
    const int n = H.n;
    std::vector<std::vector<int>> adj(n);
    for (const auto& p : H.pairs) {
        adj[p.first].push_back(p.second);
        adj[p.second].push_back(p.first);
    }
    for (auto& a : adj) {
        std::sort(a.begin(), a.end());
        a.erase(std::unique(a.begin(), a.end()), a.end());
    }
    std::vector<char> done(n, 0);
    using Item = std::pair<int, int>;   // (degree, node): smallest degree, then smallest index
    std::priority_queue<Item, std::vector<Item>, std::greater<Item>> q;
    for (int v = 0; v < n; ++v) q.emplace((int)adj[v].size(), v);
    order.clear();
    later.assign(n, {});
    std::vector<int> merged;
    while (!q.empty()) {
        const Item it = q.top();
        q.pop();
        const int v = it.second;
        if (done[v] || it.first != (int)adj[v].size()) continue;   // stale entry
        done[v] = 1;
        order.push_back(v);
        later[v] = adj[v];
        // the neighbours of v become a clique
        for (int u : adj[v]) {
            merged.clear();
            std::set_union(adj[u].begin(), adj[u].end(), adj[v].begin(), adj[v].end(), std::back_inserter(merged));
            adj[u].clear();
            for (int w : merged)
                if (w != u && w != v) adj[u].push_back(w);
            q.emplace((int)adj[u].size(), u);
        }
        adj[v].clear();
        adj[v].shrink_to_fit();
    }
}

// H x = rhs by a block sparse Cholesky (right-looking, minimum-degree order)
std::vector<double> solve_cholesky(const BlockMatrix& H, const std::vector<double>& rhs)
{
    const int n = H.n;
    std::vector<int> order;
    std::vector<std::vector<int>> later;
    minimum_degree(H, order, later);
    std::vector<int> pos(n);
    for (int k = 0; k < n; ++k) pos[order[k]] = k;
    // col[v][i] = block (row later[v][i], column v)
    std::vector<std::vector<Mat3>> col(n);
    for (int v = 0; v < n; ++v) col[v].assign(later[v].size(), Mat3{});
    auto slot = [&](int v, int u) -> Mat3& {
        const auto& L = later[v];
        const auto it = std::lower_bound(L.begin(), L.end(), u);
        return col[v][it - L.begin()];
    };
    for (size_t p = 0; p < H.pairs.size(); ++p) {
        const int a = H.pairs[p].first, b = H.pairs[p].second;   // block (a, b)
        if (pos[a] < pos[b]) {
            Mat3& s = slot(a, b);   // block (b, a) = (a, b)^T
            const Mat3 t = transpose(H.off[p]);
            for (int k = 0; k < 9; ++k) s[k] += t[k];
        } else {
            Mat3& s = slot(b, a);
            for (int k = 0; k < 9; ++k) s[k] += H.off[p][k];
        }
    }
    std::vector<Mat3> D = H.diag, Lvv(n);
    for (int k = 0; k < n; ++k) {
        const int v = order[k];
        Lvv[v] = chol3(D[v]);
        auto& C = col[v];
        for (auto& B : C) B = right_solve_lt(B, Lvv[v]);   // L_uv = A_uv L_vv^{-T}
        const auto& R = later[v];
        for (size_t i = 0; i < R.size(); ++i) {
            const int u = R[i];
            sub_into(D[u], mul_nt(C[i], C[i]));
            for (size_t j = i + 1; j < R.size(); ++j) {
                const int w = R[j];
                // block (later one, earlier one) lives in the earlier one's column
                if (pos[u] < pos[w])
                    sub_into(slot(u, w), mul_nt(C[j], C[i]));
                else
                    sub_into(slot(w, u), mul_nt(C[i], C[j]));
            }
        }
    }
    // L y = rhs, then L^T x = y
    std::vector<Vec3> y(n);
    for (int v = 0; v < n; ++v) y[v] = Vec3{ rhs[3 * v], rhs[3 * v + 1], rhs[3 * v + 2] };
    for (int k = 0; k < n; ++k) {
        const int v = order[k];
        y[v] = lsolve(Lvv[v], y[v]);
        const auto& R = later[v];
        for (size_t i = 0; i < R.size(); ++i) {
            const Vec3 d = mulv(col[v][i], y[v]);
            for (int c = 0; c < 3; ++c) y[R[i]][c] -= d[c];
        }
    }
    for (int k = n - 1; k >= 0; --k) {
        const int v = order[k];
        Vec3 r = y[v];
        const auto& R = later[v];
        for (size_t i = 0; i < R.size(); ++i) {
            const Vec3 d = mulv_t(col[v][i], y[R[i]]);
            for (int c = 0; c < 3; ++c) r[c] -= d[c];
        }
        y[v] = ltsolve(Lvv[v], r);
    }
    std::vector<double> x((size_t)3 * n);
    for (int v = 0; v < n; ++v)
        for (int c = 0; c < 3; ++c) x[3 * v + c] = y[v][c];
    return x;
}

inline double dot(const std::vector<double>& a, const std::vector<double>& b)
{
    double s = 0.0;
    for (size_t i = 0; i < a.size(); ++i) s += a[i] * b[i];
    return s;
}

// Eigen::ConjugateGradient<SparseMatrix<double>> with its defaults (Jacobi
// preconditioner, tolerance = machine epsilon, at most 2 * cols iterations,
// zero initial guess): Eigen/src/IterativeLinearSolvers/ConjugateGradient.h
std::vector<double> solve_cg(const BlockMatrix& H, const std::vector<double>& rhs)
{
    const size_t m = rhs.size();
    std::vector<double> x(m, 0.0), invdiag(m);
    for (int v = 0; v < H.n; ++v)
        for (int c = 0; c < 3; ++c) {
            const double d = H.diag[v][4 * c];
            invdiag[3 * v + c] = (d != 0.0) ? 1.0 / d : 1.0;
        }
    const double tol = std::numeric_limits<double>::epsilon();
    const int max_iters = 2 * (int)m;
    const double rhs_norm2 = dot(rhs, rhs);
    if (rhs_norm2 == 0.0) return x;
    const double consider_as_zero = std::numeric_limits<double>::min();
    const double threshold = std::max(tol * tol * rhs_norm2, consider_as_zero);
    std::vector<double> r = rhs;   // rhs - H * 0
    double r_norm2 = dot(r, r);
    if (r_norm2 < threshold) return x;
    std::vector<double> p(m), z(m);
    for (size_t i = 0; i < m; ++i) p[i] = invdiag[i] * r[i];
    double abs_new = dot(r, p);
    for (int i = 0; i < max_iters; ++i) {
        const std::vector<double> t = H.apply(p);
        const double alpha = abs_new / dot(p, t);
        for (size_t k = 0; k < m; ++k) x[k] += alpha * p[k];
        for (size_t k = 0; k < m; ++k) r[k] -= alpha * t[k];
        r_norm2 = dot(r, r);
        if (r_norm2 < threshold) break;
        for (size_t k = 0; k < m; ++k) z[k] = invdiag[k] * r[k];
        const double abs_old = abs_new;
        abs_new = dot(r, z);
        const double beta = abs_new / abs_old;
        for (size_t k = 0; k < m; ++k) p[k] = z[k] + beta * p[k];
    }
    return x;
}

inline double quad(const Vec3& e, const Matrix3d& L)   // e^T Lambda e
{
    const Vec3 t = mulv_t(L.m, e);
    return t[0] * e[0] + t[1] * e[1] + t[2] * e[2];
}

}  // namespace

// ---------------------------------------------------------------------------
// PoseGraphOptimizerLM (C/mapping/pose_graph_optimizer_lm.cpp)
// ---------------------------------------------------------------------------
void PoseGraphOptimizerLM::ComputeErrorFunction(const RobotPose2D<double>& s, const RobotPose2D<double>& e,
                                                const RobotPose2D<double>& z, std::array<double, 3>& err) const
{
    // :283-299: e_ij = h(c_i, c_j) - z_ij, angle normalised
    const RobotPose2D<double> rel = InverseCompound(s, e);
    err = { rel.mX - z.mX, rel.mY - z.mY, NormalizeAngle(rel.mTheta - z.mTheta) };
}

double PoseGraphOptimizerLM::ComputeTotalError(const std::vector<PoseGraph::Node>& nodes,
                                               const std::vector<PoseGraph::Edge>& edges) const
{
    double total = 0.0;
    for (const auto& edge : edges) {
        Vec3 e;
        ComputeErrorFunction(nodes.at(edge.StartNodeIndex()).Pose(), nodes.at(edge.EndNodeIndex()).Pose(),
                             edge.RelativePose(), e);
        total += mLossFunction->Loss(quad(e, edge.InformationMatrix()));
    }
    return total;
}

void PoseGraphOptimizerLM::OptimizeStep(std::vector<PoseGraph::Node>& nodes,
                                        const std::vector<PoseGraph::Edge>& edges)
{
    const int n = (int)nodes.size();
    BlockMatrix H;
    H.reset(n);
    std::vector<double> b((size_t)3 * n, 0.0);
    for (const auto& edge : edges) {
        const int si = edge.StartNodeIndex(), ei = edge.EndNodeIndex();
        const RobotPose2D<double>& sp = nodes.at(si).Pose();
        const RobotPose2D<double>& ep = nodes.at(ei).Pose();
        // ComputeErrorJacobians (:224-280)
        const double dx = ep.mX - sp.mX, dy = ep.mY - sp.mY;
        double sinT, cosT;
        sincos(sp.mTheta, &sinT, &cosT);
        const double ex = -sinT * dx + cosT * dy, ey = -cosT * dx - sinT * dy;
        const Mat3 Js{ -cosT, -sinT, ex, sinT, -cosT, ey, 0.0, 0.0, -1.0 };
        const Mat3 Je{ cosT, sinT, 0.0, -sinT, cosT, 0.0, 0.0, 0.0, 1.0 };
        Vec3 e;
        ComputeErrorFunction(sp, ep, edge.RelativePose(), e);
        // robust weight of e^T Lambda e (:113-115)
        const double w = mLossFunction->Weight(quad(e, edge.InformationMatrix()));
        Mat3 W;
        for (int k = 0; k < 9; ++k) W[k] = w * edge.InformationMatrix().m[k];
        const Mat3 JsW = mul_tn(Js, W), JeW = mul_tn(Je, W);
        const Mat3 JsWJs = mul(JsW, Js), JsWJe = mul(JsW, Je), JeWJe = mul(JeW, Je);
        // the four blocks (:136-157): (s, s), (e, e), (s, e), (e, s) = (s, e)^T
        if (si == ei) {
            for (int k = 0; k < 9; ++k) H.diag[si][k] += JsWJs[k];
            for (int k = 0; k < 9; ++k) H.diag[si][k] += JeWJe[k];
            const Mat3 t = transpose(JsWJe);
            for (int k = 0; k < 9; ++k) H.diag[si][k] += JsWJe[k];
            for (int k = 0; k < 9; ++k) H.diag[si][k] += t[k];
        } else {
            for (int k = 0; k < 9; ++k) H.diag[si][k] += JsWJs[k];
            for (int k = 0; k < 9; ++k) H.diag[ei][k] += JeWJe[k];
            H.add_off(si, ei, JsWJe);
        }
        const Vec3 bs = mulv(JsW, e), be = mulv(JeW, e);   // :160-161
        for (int k = 0; k < 3; ++k) {
            b[3 * si + k] += bs[k];
            b[3 * ei + k] += be[k];
        }
    }
    // :167-172: fix node 0 with 1e9, then lambda on every diagonal entry
    if (n > 0)
        for (int k = 0; k < 3; ++k) H.diag[0][4 * k] += 1e9;
    for (int v = 0; v < n; ++v)
        for (int k = 0; k < 3; ++k) H.diag[v][4 * k] += mLambda;
    std::vector<double> rhs(b.size());
    for (size_t i = 0; i < b.size(); ++i) rhs[i] = -b[i];
    const std::vector<double> delta =
        (mSolverType == SolverType::SparseCholesky) ? solve_cholesky(H, rhs) : solve_cg(H, rhs);
    for (int i = 0; i < n; ++i) {   // :209-217
        const RobotPose2D<double>& p = nodes.at(i).Pose();
        nodes.at(i).Pose() =
            RobotPose2D<double>(p.mX + delta[3 * i], p.mY + delta[3 * i + 1], p.mTheta + delta[3 * i + 2]);
    }
}

void PoseGraphOptimizerLM::Optimize(std::vector<PoseGraph::Node>& nodes, const std::vector<PoseGraph::Edge>& edges)
{
    for (const auto& edge : edges)
        if (edge.StartNodeIndex() < 0 || edge.StartNodeIndex() >= (int)nodes.size() || edge.EndNodeIndex() < 0 ||
            edge.EndNodeIndex() >= (int)nodes.size())
            throw std::out_of_range("PoseGraphOptimizerLM: edge node index out of range");   // the reference's .at()
    double prevTotalError = std::numeric_limits<double>::max();
    double totalError = std::numeric_limits<double>::max();
    int numOfIterations = 0;
    while (true) {
        OptimizeStep(nodes, edges);
        totalError = ComputeTotalError(nodes, edges);
        if (++numOfIterations >= mNumOfIterationsMax || std::fabs(prevTotalError - totalError) < mErrorTolerance)
            break;
        if (totalError < prevTotalError)
            mLambda *= 0.5;
        else
            mLambda *= 2.0;
        prevTotalError = totalError;
    }
    mLastIterations = numOfIterations;
    mLastTotalError = totalError;
}

}  // namespace Mapping
}  // namespace Hip
}  // namespace MyLidarGraphSlam
