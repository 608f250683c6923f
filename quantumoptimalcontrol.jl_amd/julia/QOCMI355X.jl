# QOCMI355X.jl — ccall shim that routes QuantumOptimalControl.jl's PWC GRAPE hot path to
# libqoc_mi355x.so (C ABI: include/qoc.h).  Nothing else in the reference changes: the Ipopt
# callbacks (examples/ipopt_callbacks_exp.jl) keep calling `QuantumOptimalControl.propagate`
# and `grape_sensitivity`; only the `setup_grape_cache` line constructs an `MI355XCache`.
#
#   cache = QOCMI355X.setup_grape_cache(A0Δt, complex(x0), (2, segment_count))
#   x     = QuantumOptimalControl.propagate(A0Δt, [A1Δt, A2Δt], u, x0, cache)      # method below
#   dJdu  = QuantumOptimalControl.grape_sensitivity(A0Δt, [A1Δt, A2Δt], dJfinal_dx, cache.u, x0, cache;
#                                                   dUkdp_order=3, dL_dx=dL_dx)
#
# Memory layout needs no conversion: Matrix{ComplexF64} is column-major interleaved (re, im),
# exactly the ABI's layout; u / dJdu are Matrix{Float64} (nu x Nt).
module QOCMI355X

import QuantumOptimalControl
using LinearAlgebra: tr
const QOC = QuantumOptimalControl

const libqoc = get(ENV, "QOC_MI355X_LIB", joinpath(@__DIR__, "..", "qoc_amd", "libqoc_mi355x.so"))

const QOC_FP64 = Cint(0)
const QOC_COST_TRACE = Cint(0)
const QOC_COST_ZCAL = Cint(1)
const QOC_COST_EXTERNAL = Cint(2)
const QOC_ERR_STALE = Cint(-3)

qoc_error(ctx) = unsafe_string(ccall((:qoc_last_error, libqoc), Cstring, (Ptr{Cvoid},), ctx))

function check(rc, ctx)
    rc == 0 && return nothing
    # the reference raises error(...) at src/gradient_computations.jl:37-39 and :84-87
    error(qoc_error(ctx))
end

mutable struct MI355XCache
    ctx::Ptr{Cvoid}
    N::Int
    m::Int
    nu::Int
    Nt::Int
    u::Matrix{Float64}
    dJdu::Matrix{Float64}
    gen::UInt64        # hash of the generators last uploaded
    x0::UInt64
    function MI355XCache(ctx, N, m, nu, Nt)
        c = new(ctx, N, m, nu, Nt, zeros(nu, Nt), zeros(nu, Nt), 0, 0)
        finalizer(c) do c
            c.ctx != C_NULL && ccall((:qoc_destroy, libqoc), Cvoid, (Ptr{Cvoid},), c.ctx)
            c.ctx = C_NULL
        end
        return c
    end
end

"""
    setup_grape_cache(A0, x0, u_size; device=0, compress=nothing)

GPU-resident replacement of `QuantumOptimalControl.setup_grape_cache`
(src/gradient_computations.jl:79-96).  Errors on a dimension mismatch like the reference.
`compress = v` takes the reference's `compress_states` spec (src/utils.jl:96-109, 1-based, e.g.
`((1:2:27, [1,4]), (2:2:26, [2,3]))`): the kernels then run on the packed columns while `x`, `dJfinal_dx`
and `dL_dx` keep the caller's N x m layout (qoc_set_compression).
"""
function setup_grape_cache(A0, x0, u_size; device::Integer=0, compress=nothing)
    size(x0, 1) == size(A0, 1) || error("Error when creating cache, A0 and x0 have incompatiable dimensions")
    nu, Nt = u_size
    ref = Ref{Ptr{Cvoid}}(C_NULL)
    rc = ccall((:qoc_create, libqoc), Cint,
               (Ref{Ptr{Cvoid}}, Cint, Cint, Cint, Cint, Cint, Cint, Cint),
               ref, device, size(A0, 1), size(x0, 2), nu, Nt, 1, QOC_FP64)
    check(rc, C_NULL)
    c = MI355XCache(ref[], size(A0, 1), size(x0, 2), nu, Nt)
    check(ccall((:qoc_set_cost, libqoc), Cint, (Ptr{Cvoid}, Cint, Ptr{ComplexF64}, Cdouble),
                c.ctx, QOC_COST_EXTERNAL, C_NULL, 1.0), c.ctx)
    compress === nothing || set_compression!(c, compress)
    return c
end

function set_compression!(c::MI355XCache, v)
    (r1, c1), (r2, c2) = v
    l = [Cint.(collect(a) .- 1) for a in (r1, c1, r2, c2)]   # 0-based
    check(ccall((:qoc_set_compression, libqoc), Cint,
                (Ptr{Cvoid}, Ptr{Cint}, Cint, Ptr{Cint}, Cint, Ptr{Cint}, Cint, Ptr{Cint}, Cint),
                c.ctx, l[1], length(l[1]), l[2], length(l[2]), l[3], length(l[3]), l[4], length(l[4])), c.ctx)
end

function upload!(c::MI355XCache, A0, A, x0)
    h = hash((A0, A))
    if h != c.gen
        A0c = Matrix{ComplexF64}(A0)
        Ac = [Matrix{ComplexF64}(a) for a in A]
        ptrs = [pointer(a) for a in Ac]
        GC.@preserve A0c Ac ptrs begin
            check(ccall((:qoc_set_generators, libqoc), Cint, (Ptr{Cvoid}, Ptr{ComplexF64}, Ptr{Ptr{ComplexF64}}),
                        c.ctx, A0c, ptrs), c.ctx)
        end
        c.gen = h
    end
    hx = hash(x0)
    if hx != c.x0
        x0c = Matrix{ComplexF64}(reshape(x0, size(x0, 1), :))
        GC.@preserve x0c check(ccall((:qoc_set_x0, libqoc), Cint, (Ptr{Cvoid}, Ptr{ComplexF64}, Cint),
                                     c.ctx, x0c, 0), c.ctx)
        c.x0 = hx
    end
end

"""States of the last propagate, fetched lazily (the reference returns cache.x, Nt+1 matrices)."""
struct LazyStates <: AbstractVector{Matrix{ComplexF64}}
    c::MI355XCache
end
Base.size(s::LazyStates) = (s.c.Nt + 1,)
function Base.getindex(s::LazyStates, k::Int)
    out = Matrix{ComplexF64}(undef, s.c.N, s.c.m)
    check(ccall((:qoc_get_states, libqoc), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{ComplexF64}),
                s.c.ctx, 0, k - 1, out), s.c.ctx)
    return out
end

function Base.getproperty(c::MI355XCache, s::Symbol)
    s === :x && return LazyStates(c)
    return getfield(c, s)
end

# propagate (src/gradient_computations.jl:2-32) on the GPU
function QOC.propagate(A0, A::Vector{<:AbstractMatrix}, u, x0, cache::MI355XCache)
    upload!(cache, A0, A, x0)
    cache.u .= u                              # :12, kept for the stale-u check
    J = Ref{Cdouble}(0.0)
    check(ccall((:qoc_propagate, libqoc), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ref{Cdouble}),
                cache.ctx, cache.u, J), cache.ctx)
    return cache.x
end

# grape_sensitivity (src/gradient_computations.jl:35-77) on the GPU; the closure dJfinal_dx is
# evaluated here at x[end] and handed over as λ_{Nt+1} (QOC_COST_EXTERNAL).
function QOC.grape_sensitivity(A0, A::Vector{<:AbstractMatrix}, dJfinal_dx, u, x0, cache::MI355XCache;
                               dUkdp_order=3, dL_dx=nothing)
    # setup_state_penalty's gradient runs on the GPU; nothing clears a penalty left by an earlier call
    # (:47-57 add nothing then); any other closure is evaluated here on every state and the GPU adds
    # dL_dx(x[k]) to λ[k] (qoc_set_costate_source)
    set_penalty!(cache, dL_dx isa PenaltyGrad ? dL_dx : nothing)
    src = nothing
    if !(dL_dx === nothing || dL_dx isa PenaltyGrad)
        xs = cache.x
        src = Array{ComplexF64}(undef, cache.N, cache.m, cache.Nt + 1)
        for k in 1:cache.Nt+1
            src[:, :, k] .= dL_dx(xs[k])
        end
        GC.@preserve src check(ccall((:qoc_set_costate_source, libqoc), Cint, (Ptr{Cvoid}, Ptr{ComplexF64}),
                                     cache.ctx, src), cache.ctx)
    end
    λf = Matrix{ComplexF64}(dJfinal_dx(cache.x[end]))
    rc = ccall((:qoc_grape_sensitivity, libqoc), Cint,
               (Ptr{Cvoid}, Ptr{Float64}, Cint, Ptr{ComplexF64}, Ptr{Float64}),
               cache.ctx, Matrix{Float64}(u), dUkdp_order, λf, cache.dJdu)
    src === nothing || ccall((:qoc_set_costate_source, libqoc), Cint, (Ptr{Cvoid}, Ptr{ComplexF64}), cache.ctx, C_NULL)
    check(rc, cache.ctx)   # QOC_ERR_STALE -> "Cache data from other control signal u"
    return cache.dJdu
end

function set_penalty!(cache::MI355XCache, dL_dx)
    if dL_dx isa PenaltyGrad
        P = Cint.(dL_dx.P .- 1); C = Cint.(dL_dx.C .- 1)
        check(ccall((:qoc_set_state_penalty, libqoc), Cint,
                    (Ptr{Cvoid}, Ptr{Cint}, Cint, Ptr{Cint}, Cint, Cdouble),
                    cache.ctx, P, length(P), C, length(C), dL_dx.μ), cache.ctx)
    else
        check(ccall((:qoc_set_state_penalty, libqoc), Cint,
                    (Ptr{Cvoid}, Ptr{Cint}, Cint, Ptr{Cint}, Cint, Cdouble),
                    cache.ctx, C_NULL, 0, C_NULL, 0, 0.0), cache.ctx)
    end
end

"""Trace infidelity J = 1 - |tr(X'x)|^2/n^2 and its gradient (src/penalty_fcns.jl:15-24), tagged so that the
GPU path can evaluate them on the device; on host they behave like the reference's closures."""
struct TraceJ
    Xt::Matrix{ComplexF64}
    n::Float64
end
struct TraceGrad
    Xt::Matrix{ComplexF64}
    n::Float64
end
(f::TraceJ)(x) = 1 - abs2(tr(f.Xt' * x)) / f.n^2
(g::TraceGrad)(x) = (-2 * tr(g.Xt' * x) / g.n^2) .* g.Xt
tr(A) = sum(A[i, i] for i in 1:minimum(size(A)))
setup_infidelity(x_target, n=size(x_target, 2)) =
    (TraceJ(Matrix{ComplexF64}(x_target), n), TraceGrad(Matrix{ComplexF64}(x_target), n))

"""z-calibrated infidelity (src/penalty_fcns.jl:27-42): the reference's closures, tagged for the device."""
struct ZCalJ
    Xt::Matrix{ComplexF64}
    J::Any
end
struct ZCalGrad
    Xt::Matrix{ComplexF64}
    dJ::Any
end
(f::ZCalJ)(x) = f.J(x)
(g::ZCalGrad)(x) = g.dJ(x)
function setup_infidelity_zcalibrated(x_target)
    J, dJ = QOC.setup_infidelity_zcalibrated(x_target)
    return ZCalJ(Matrix{ComplexF64}(x_target), J), ZCalGrad(Matrix{ComplexF64}(x_target), dJ)
end

# the reference's "no penalty" pair (examples/zz_coupling_ipopt_exp.jl:46: Returns(0), x -> 0*x)
no_penalty(L) = L === nothing || (L isa Base.Returns && iszero(L.value))

"""Guard-state penalty whose gradient the GPU applies at every slice (src/penalty_fcns.jl:1-11)."""
struct PenaltyGrad
    P::Vector{Int}
    C::Vector{Int}
    μ::Float64
end
(g::PenaltyGrad)(x) = (d = zeros(eltype(x), size(x)); d[g.P, g.C] .= 2g.μ .* x[g.P, g.C]; d)
function setup_state_penalty(inds_penalty, inds_css, μ)
    L, _ = QOC.setup_state_penalty(inds_penalty, inds_css, μ)
    return L, PenaltyGrad(collect(inds_penalty), collect(inds_css), Float64(μ))
end

# x_target / n given with untagged closures: they must be the trace infidelity of x_target (the reference's
# setup_infidelity(x_target, n), src/penalty_fcns.jl:15-24), checked on a probe state.
function check_trace_closures(Jfinal, dJfinal_dx, Xt, nn)
    xp = Xt .+ 0.1 .* cis.(reshape(1:length(Xt), size(Xt)))
    Ω = tr(Xt' * xp)
    Jw, dJw = 1 - abs2(Ω) / nn^2, -2Ω / nn^2 .* Xt
    ok = isapprox(Jfinal(xp), Jw; rtol=1e-12, atol=1e-14) &&
         isapprox(dJfinal_dx(xp), dJw; rtol=1e-12, atol=1e-14)
    ok || error("x_target given but (Jfinal, dJfinal_dx) are not setup_infidelity(x_target, n): pass the " *
                "closures without x_target (host-evaluated cost) or use QOCMI355X.setup_infidelity")
    return nothing
end

"""
    setup_ipopt_callbacks(A0Δt, A1Δt, A2Δt, x0, u_prototype, (Jfinal, dJfinal_dx), (L, dL_dx), B; x_target, n)

GPU version of examples/ipopt_callbacks_exp.jl:1-54: f = Jfinal(x[end]) + sum(L, x) and f_grad = B' dJdu'.
As in the reference, f only propagates (Ipopt's line-search evaluations pay no gradient) and f_grad runs the
sensitivity of the coefficients f last saw, re-propagating first if Ipopt asks for the gradient of new ones.
With the tagged costs of this module (setup_infidelity / setup_infidelity_zcalibrated) and penalty
(setup_state_penalty, or the reference's disabled Returns(0) pair) both run on the device
(`qoc_propagate_spline`, `qoc_sensitivity_spline`).  Any other cost closure is evaluated on
the host at x[end] and handed over as λ_{Nt+1} (QOC_COST_EXTERNAL), exactly as the reference's f / f_grad do;
any other penalty pair is evaluated on the host too: sum(L, x) in f, and dL_dx(x[k]) for every slice added to
the co-states on the device (qoc_set_costate_source).  g / g_jac are the reference's norm constraints.
Returns the same tuple.
"""
function setup_ipopt_callbacks(A0Δt, A1Δt, A2Δt, x0, u_prototype, (Jfinal, dJfinal_dx), (L, dL_dx), B;
                               x_target=nothing, n=nothing)
    nu = size(u_prototype, 1)
    ng = 2
    nx = length(x0)
    nsplines = size(B, 2)
    nc = nu * nsplines
    Nt = size(B, 1)
    ref = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:qoc_create, libqoc), Cint, (Ref{Ptr{Cvoid}}, Cint, Cint, Cint, Cint, Cint, Cint, Cint),
                ref, 0, size(A0Δt, 1), size(x0, 2), nu, Nt, 1, QOC_FP64), C_NULL)
    cache = MI355XCache(ref[], size(A0Δt, 1), size(x0, 2), nu, Nt)
    A = [A1Δt, A2Δt][1:nu]
    upload!(cache, A0Δt, A, complex(x0))
    # penalty: the device applies setup_state_penalty's; the reference's disabled pair adds nothing; any
    # other (L, dL_dx) takes the host path below (sum(L, x) on the host, dL_dx through the co-state source)
    device_penalty = dL_dx isa PenaltyGrad || no_penalty(L)
    set_penalty!(cache, dL_dx isa PenaltyGrad ? dL_dx : nothing)
    # cost: on the device when tagged, else the caller's closures on the host.  The x_target / n keywords name the
    # trace infidelity for callers that pass the reference's own (untagged) setup_infidelity(x_target, n)
    # closures; closures that are not that cost are an error rather than silently replaced by it.
    if Jfinal isa TraceJ || (x_target !== nothing && !(Jfinal isa ZCalJ))
        Xt = Jfinal isa TraceJ ? Jfinal.Xt : Matrix{ComplexF64}(x_target)
        nn = Jfinal isa TraceJ ? Jfinal.n : (n === nothing ? size(Xt, 2) : n)
        Jfinal isa TraceJ || check_trace_closures(Jfinal, dJfinal_dx, Xt, nn)
        kind = QOC_COST_TRACE
    elseif Jfinal isa ZCalJ
        Xt, nn, kind = Jfinal.Xt, 4.0, QOC_COST_ZCAL
    else
        Xt, nn, kind = Matrix{ComplexF64}(undef, 0, 0), 1.0, QOC_COST_EXTERNAL
    end
    check(ccall((:qoc_set_cost, libqoc), Cint, (Ptr{Cvoid}, Cint, Ptr{ComplexF64}, Cdouble),
                cache.ctx, kind, kind == QOC_COST_EXTERNAL ? C_NULL : Xt, nn), cache.ctx)
    Bm = Matrix{Float64}(B)
    check(ccall((:qoc_set_spline_basis, libqoc), Cint, (Ptr{Cvoid}, Ptr{Float64}, Cint),
                cache.ctx, Bm, nsplines), cache.ctx)
    c_prev = fill(NaN, nc)
    J = Ref{Cdouble}(0.0)
    dJdc = zeros(nc)
    on_device = kind != QOC_COST_EXTERNAL && device_penalty
    # f: examples/ipopt_callbacks_exp.jl:11-19 — spline map, propagate, cost; no sensitivity
    propagate!(c) = if on_device
        check(ccall((:qoc_propagate_spline, libqoc), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ref{Cdouble}),
                    cache.ctx, c, J), cache.ctx)
    else
        u = Matrix(transpose(Bm * reshape(c, nsplines, nu)))
        x = QOC.propagate(A0Δt, A, u, x0, cache)
        J[] = Jfinal(x[end]) + (no_penalty(L) ? 0.0 : sum(L, x))
    end
    # f_grad: :21-31 — the sensitivity of the last propagated c, mapped to the coefficients (B' dJdu')
    sensitivity!(c) = if on_device
        check(ccall((:qoc_sensitivity_spline, libqoc), Cint, (Ptr{Cvoid}, Ptr{Float64}, Cint, Ptr{Float64}),
                    cache.ctx, c, 3, dJdc), cache.ctx)
    else
        dJdu = QOC.grape_sensitivity(A0Δt, A, dJfinal_dx, cache.u, x0, cache; dUkdp_order=3, dL_dx=dL_dx)
        dJdc .= (Bm' * transpose(dJdu))[:]
    end
    f = function (c::Vector{Float64})
        c_prev .= c
        propagate!(c)
        J[]
    end
    f_grad = function (c, f_grad_out)
        if c_prev != c  # Ipopt asked for the gradient first (:22-25)
            c_prev .= c
            propagate!(c)
        end
        sensitivity!(c)
        f_grad_out .= dJdc
    end
    g_oop = function (c)
        cm = reshape(c, nsplines, nu)
        [sqrt(sum(abs2, cm)); sqrt(sum(abs2, diff(cm, dims=1)))]
    end
    g = (c, g_out) -> (g_out .= g_oop(c))
    function g_jac(c, mode, rows, cols, g_jac_out)
        if mode == :Structure
            cols .= kron(ones(ng), 1:nc)
            rows .= kron(1:ng, ones(nc))
        else
            cm = reshape(c, nsplines, nu)
            g0, g1 = g_oop(c)
            D = zeros(nsplines + 1, nu)
            D[2:nsplines, :] .= diff(cm, dims=1)
            j1 = (D[1:nsplines, :] .- D[2:end, :])[:]
            g_jac_out .= [g0 > 0 ? c ./ g0 : zero(c); g1 > 0 ? j1 ./ g1 : zero(j1)]
        end
    end
    f, g, f_grad, g_jac, nu, ng, nx, nc, cache
end

end # module
