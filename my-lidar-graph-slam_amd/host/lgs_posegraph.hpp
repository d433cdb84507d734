// lgs_posegraph.hpp -- the pose graph and its Levenberg-Marquardt optimizer
// (SURVEY.md §8(f) f4), host C++ with the reference's class names:
//
//   reference (H/ = include/my_lidar_graph_slam/, C/ = src/my_lidar_graph_slam/)   here
//   Mapping::PoseGraph::Node / Edge (H/mapping/pose_graph.hpp:70-170)              PoseGraph::Node / Edge
//   Mapping::LossFunction + LossSquared/Huber/Cauchy/Fair/GemanMcClure/Welsch/DCS
//     (H/mapping/robust_loss_function.hpp, C/mapping/robust_loss_function.cpp:17-188)  same names
//   Mapping::PoseGraphOptimizerLM (H/mapping/pose_graph_optimizer_lm.hpp:34-119,
//     C/mapping/pose_graph_optimizer_lm.cpp:13-338)                               PoseGraphOptimizerLM
//
// The pose graph is a sparse nonlinear least-squares problem over 3-vectors
// (Sparse Pose Adjustment): a few thousand nodes, each linked to its
// neighbours and a handful of loop edges.  It is not a grid workload and its
// factorisation is a chain of small dependent 3x3 block operations, so it
// stays on the host: the reference's Eigen SimplicialLDLT is
// replaced by a block (3x3) sparse Cholesky with a minimum-degree node
// ordering, and Eigen's ConjugateGradient by the same Jacobi-preconditioned
// CG recurrence.  No Eigen: matrices are row-major std::array.
#pragma once

#include <array>
#include <memory>
#include <string>
#include <vector>

#include "lgs_slam_hip.hpp"

namespace MyLidarGraphSlam {
namespace Hip {
namespace Mapping {

// RobotPose2D algebra of H/pose.hpp / H/util.hpp that the optimizer uses
// (sin/cos of one argument as one glibc sincos, as GCC -O3 emits it)
RobotPose2D<double> InverseCompound(const RobotPose2D<double>& startPose, const RobotPose2D<double>& endPose);
RobotPose2D<double> Compound(const RobotPose2D<double>& startPose, const RobotPose2D<double>& diffPose);
double NormalizeAngle(double theta);   // H/util.hpp:125-135

class PoseGraph {
public:
    // H/mapping/pose_graph.hpp:70-114 (the scan pointer is reduced to what the
    // savers read from it: its timestamp)
    class Node final {
    public:
        Node(int nodeIdx, const RobotPose2D<double>& pose, double timeStamp = 0.0)
            : mIdx(nodeIdx), mPose(pose), mTimeStamp(timeStamp) {}
        int Index() const { return mIdx; }
        RobotPose2D<double>& Pose() { return mPose; }
        const RobotPose2D<double>& Pose() const { return mPose; }
        double TimeStamp() const { return mTimeStamp; }

    private:
        int mIdx;
        RobotPose2D<double> mPose;
        double mTimeStamp;
    };

    // H/mapping/pose_graph.hpp:120-170
    class Edge final {
    public:
        Edge(int startNodeIdx, int endNodeIdx, const RobotPose2D<double>& relativePose, const Matrix3d& infoMat)
            : mStartNodeIdx(startNodeIdx), mEndNodeIdx(endNodeIdx), mRelativePose(relativePose),
              mInformationMat(infoMat) {}
        int StartNodeIndex() const { return mStartNodeIdx; }
        int EndNodeIndex() const { return mEndNodeIdx; }
        const RobotPose2D<double>& RelativePose() const { return mRelativePose; }
        const Matrix3d& InformationMatrix() const { return mInformationMat; }
        bool IsOdometricConstraint() const { return mEndNodeIdx == mStartNodeIdx + 1; }
        bool IsLoopClosingConstraint() const { return !IsOdometricConstraint(); }

    private:
        int mStartNodeIdx;
        int mEndNodeIdx;
        RobotPose2D<double> mRelativePose;
        Matrix3d mInformationMat;
    };

    int AppendNode(const RobotPose2D<double>& pose, double timeStamp = 0.0);
    void AppendEdge(int startNodeIdx, int endNodeIdx, const RobotPose2D<double>& relativePose,
                    const Matrix3d& informationMat);
    const std::vector<Node>& Nodes() const { return mNodes; }
    std::vector<Node>& Nodes() { return mNodes; }
    Node& NodeAt(int nodeIdx) { return mNodes.at(nodeIdx); }
    const Node& NodeAt(int nodeIdx) const { return mNodes.at(nodeIdx); }
    const std::vector<Edge>& Edges() const { return mEdges; }

private:
    std::vector<Node> mNodes;
    std::vector<Edge> mEdges;
};

// C/mapping/robust_loss_function.cpp: Loss(t) = rho(t), Weight(t) = rho'(t)
// of a squared error t >= 0
class LossFunction {
public:
    virtual ~LossFunction() = default;
    virtual double Loss(double squaredError) const = 0;
    virtual double Weight(double squaredError) const = 0;
};
using LossFunctionPtr = std::shared_ptr<LossFunction>;

class LossSquared final : public LossFunction {   // H/mapping/robust_loss_function.hpp:36-50
public:
    double Loss(double t) const override { return t; }
    double Weight(double) const override { return 1.0; }
};

#define LGS_SCALED_LOSS(Name)                                   \
    class Name final : public LossFunction {                    \
    public:                                                     \
        explicit Name(double scale) : mScale(scale) {}          \
        double Loss(double squaredError) const override;        \
        double Weight(double squaredError) const override;      \
                                                                \
    private:                                                    \
        double mScale;                                          \
    };
LGS_SCALED_LOSS(LossHuber)          // :17-43
LGS_SCALED_LOSS(LossCauchy)         // :45-72
LGS_SCALED_LOSS(LossFair)           // :74-103
LGS_SCALED_LOSS(LossGemanMcClure)   // :105-134
LGS_SCALED_LOSS(LossWelsch)         // :136-162
LGS_SCALED_LOSS(LossDCS)            // :164-188
#undef LGS_SCALED_LOSS

// kind: 0 Huber, 1 Cauchy, 2 Fair, 3 GemanMcClure, 4 Welsch, 5 DCS, 6 Squared
// (the launcher's CreateLossFunction names, C/slam_launcher.cpp:603-624)
LossFunctionPtr CreateLossFunction(int kind, double scale);

class PoseGraphOptimizerLM final {
public:
    enum class SolverType { SparseCholesky, ConjugateGradient };

    PoseGraphOptimizerLM(SolverType solverType, int numOfIterationsMax, double errorTolerance, double initialLambda,
                         LossFunctionPtr lossFunction)
        : mSolverType(solverType), mNumOfIterationsMax(numOfIterationsMax), mErrorTolerance(errorTolerance),
          mLambda(initialLambda), mLossFunction(std::move(lossFunction)) {}

    // C/mapping/pose_graph_optimizer_lm.cpp:13-65.  The damping factor is a
    // member and carries over to the next call, as in the reference.
    void Optimize(std::vector<PoseGraph::Node>& poseGraphNodes, const std::vector<PoseGraph::Edge>& poseGraphEdges);
    // :283-299
    void ComputeErrorFunction(const RobotPose2D<double>& startNodePose, const RobotPose2D<double>& endNodePose,
                              const RobotPose2D<double>& edgeRelPose, std::array<double, 3>& errorVec) const;
    // :302-338
    double ComputeTotalError(const std::vector<PoseGraph::Node>& poseGraphNodes,
                             const std::vector<PoseGraph::Edge>& poseGraphEdges) const;

    double Lambda() const { return mLambda; }
    int LastIterations() const { return mLastIterations; }
    double LastTotalError() const { return mLastTotalError; }

private:
    // :68-220: H and b from every edge, the 1e9 anchor on node 0, lambda on the
    // diagonal, then H delta = -b; poses += delta
    void OptimizeStep(std::vector<PoseGraph::Node>& poseGraphNodes, const std::vector<PoseGraph::Edge>& poseGraphEdges);

    SolverType mSolverType;
    int mNumOfIterationsMax;
    double mErrorTolerance;
    double mLambda;
    LossFunctionPtr mLossFunction;
    int mLastIterations = 0;
    double mLastTotalError = 0.0;
};

}  // namespace Mapping
}  // namespace Hip
}  // namespace MyLidarGraphSlam
