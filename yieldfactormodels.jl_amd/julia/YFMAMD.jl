# Julia @ccall binding of libyfm_hip.so (include/yfm.h). Not executable in this image (no julia).
# See INTEGRATION.md for the drop-in get_loss / predict / get_loss_array / estimate_steps! methods.
module YFMAMD
const LIB = get(ENV, "YFM_LIB", joinpath(@__DIR__, "..", "yfm_amd", "libyfm_hip.so"))

const YFM_MODEL_DNS, YFM_MODEL_TVL, YFM_MODEL_GNS5 = Cint(0), Cint(1), Cint(2)
const UNCONSTRAINED, CONSTRAINED = Cint(0), Cint(1)
const PREC_CERTIFIED, PREC_FP64 = Cint(0), Cint(1)     # TVλ arithmetic (yfm_set_precision)

struct YFMError <: Exception; code::Cint; msg::String; end
check(rc) = rc == 0 || throw(YFMError(rc, unsafe_string(@ccall LIB.yfm_last_error()::Cstring)))

mutable struct Context
    ptr::Ptr{Cvoid}
    # The panel last uploaded, held by reference: identity (===) then means "this very array",
    # and holding it keeps the GC from freeing it and handing its address to a later slice
    # (an objectid comparison could match a new array at a reused address).  A panel changed
    # IN PLACE still compares equal: call set_panel! explicitly after mutating it.
    panel::Union{Nothing,Matrix{Float64}}
    maturities::Vector{Float64}
    function Context(device::Integer = 0)
        p = @ccall LIB.yfm_create(Cint(device)::Cint)::Ptr{Cvoid}
        p == C_NULL && throw(YFMError(-2, unsafe_string(@ccall LIB.yfm_last_error()::Cstring)))
        ctx = new(p, nothing, Float64[])
        finalizer(c -> @ccall(LIB.yfm_destroy(c.ptr::Ptr{Cvoid})::Cvoid), ctx)
    end
end
const CTX = Ref{Context}()
ctx() = isassigned(CTX) ? CTX[] : (CTX[] = Context(0))

function set_panel!(c::Context, data::Matrix{Float64}, maturities::Vector{Float64})
    N, T = size(data)                       # N×T column-major, as load_data returns it
    GC.@preserve data maturities check(@ccall LIB.yfm_set_panel(c.ptr::Ptr{Cvoid}, data::Ptr{Cdouble},
        Cint(N)::Cint, Cint(T)::Cint, maturities::Ptr{Cdouble})::Cint)
    c.panel = data
    c.maturities = copy(maturities)
    c
end

function ensure_panel!(model, data::Matrix{Float64})
    c = ctx()
    m = Vector{Float64}(model.base.maturities)
    (c.panel === data && c.maturities == m) || set_panel!(c, data, m)
    c
end

"Select the TVλ arithmetic: PREC_CERTIFIED (default, double-double) or PREC_FP64."
set_precision!(mode::Integer; c::Context = ctx()) = check(@ccall LIB.yfm_set_precision(c.ptr::Ptr{Cvoid},
                                                                                      Cint(mode)::Cint)::Cint)

"A P×B matrix in page-locked host memory (yfm_alloc_host): θ batches built in it reach the GPU by DMA."
function pinned_matrix(P::Integer, B::Integer)
    p = @ccall LIB.yfm_alloc_host((P * B * sizeof(Float64))::Csize_t)::Ptr{Cvoid}
    p == C_NULL && throw(YFMError(-2, unsafe_string(@ccall LIB.yfm_last_error()::Cstring)))
    A = unsafe_wrap(Array, Ptr{Float64}(p), (P, B); own = false)
    finalizer(_ -> @ccall(LIB.yfm_free_host(p::Ptr{Cvoid})::Cint), A)
    A
end

kind(::YieldFactorModels.AbstractDNSModel) = YFM_MODEL_DNS
kind(::YieldFactorModels.AbstractTVλDNSModel) = YFM_MODEL_TVL
tuse_ptr(T_use) = T_use === nothing ? C_NULL : pointer(T_use)

"Batched loglik: Θ is P×B (one candidate per column).  space: UNCONSTRAINED (compute_loss input) or CONSTRAINED (set_params! input)."
function loglik_batch(model, data::Matrix{Float64}, Θ::Matrix{Float64}; space = UNCONSTRAINED,
                      T_use::Union{Nothing,Vector{Cint}} = nothing)
    c = ensure_panel!(model, data)
    P, B = size(Θ)
    out = Vector{Float64}(undef, B)
    GC.@preserve Θ out T_use check(@ccall LIB.yfm_loglik_batch(c.ptr::Ptr{Cvoid}, kind(model)::Cint, space::Cint,
        Θ::Ptr{Cdouble}, Cint(P)::Cint, Cint(B)::Cint, tuse_ptr(T_use)::Ptr{Cint}, out::Ptr{Cdouble})::Cint)
    out                                        # +loglik per column; -Inf / NaN as documented in yfm.h
end

"Batched predict (filter.jl:250-282) on hcat(data[:, 1:T_use[b]], NaN × (horizon−1)); arrays get a trailing batch axis."
function predict_batch(model, data::Matrix{Float64}, Θc::Matrix{Float64}; horizon::Integer = 1,
                       T_use::Union{Nothing,Vector{Cint}} = nothing)
    c = ensure_panel!(model, data)
    P, B = size(Θc)
    N, T = size(data)
    M = @ccall LIB.yfm_state_dim(kind(model)::Cint)::Cint
    L = @ccall LIB.yfm_gamma_dim(kind(model)::Cint)::Cint
    ncol = T + horizon - 1
    preds, fl1, fl2 = (Array{Float64}(undef, N, ncol, B) for _ in 1:3)
    factors = Array{Float64}(undef, M, ncol, B)
    states = Array{Float64}(undef, L, ncol, B)
    GC.@preserve Θc T_use preds fl1 fl2 factors states check(@ccall LIB.yfm_predict(c.ptr::Ptr{Cvoid},
        kind(model)::Cint, CONSTRAINED::Cint, Θc::Ptr{Cdouble}, Cint(P)::Cint, Cint(B)::Cint, tuse_ptr(T_use)::Ptr{Cint},
        Cint(horizon)::Cint, preds::Ptr{Cdouble}, factors::Ptr{Cdouble}, states::Ptr{Cdouble}, fl1::Ptr{Cdouble},
        fl2::Ptr{Cdouble})::Cint)
    (preds = preds, factors = factors, states = states, factor_loadings_1 = fl1, factor_loadings_2 = fl2)
end

"get_loss_array (filter.jl:211-247) per column of Θc: (T−1)×B, −Inf rows where the reference returns −Inf."
function loss_array_batch(model, data::Matrix{Float64}, Θc::Matrix{Float64}; K::Integer = 1,
                          T_use::Union{Nothing,Vector{Cint}} = nothing)
    c = ensure_panel!(model, data)
    P, B = size(Θc)
    out = Matrix{Float64}(undef, size(data, 2) - 1, B)
    GC.@preserve Θc T_use out check(@ccall LIB.yfm_loss_array(c.ptr::Ptr{Cvoid}, kind(model)::Cint,
        CONSTRAINED::Cint, Θc::Ptr{Cdouble}, Cint(P)::Cint, Cint(B)::Cint, tuse_ptr(T_use)::Ptr{Cint}, Cint(K)::Cint,
        out::Ptr{Cdouble})::Cint)
    out
end

"R estimate_steps! chains (optimization.jl:137-312) batched on the device; starts Θ0c (constrained) on windows T_use."
function estimate_batch(model, data::Matrix{Float64}, Θ0c::Matrix{Float64}; T_use = nothing, iterations = 500,
                        g_tol = 1e-6, max_group_iters = 10, tol = 1e-8)
    c = ensure_panel!(model, data)
    P, R = size(Θ0c)
    θc, p, init = Matrix{Float64}(undef, P, R), Matrix{Float64}(undef, P, R), Matrix{Float64}(undef, P, R)
    ll, status, nev = Vector{Float64}(undef, R), Vector{Cint}(undef, R), Ref{Clonglong}(0)
    GC.@preserve Θ0c T_use θc p init ll status check(@ccall LIB.yfm_estimate(c.ptr::Ptr{Cvoid}, kind(model)::Cint,
        CONSTRAINED::Cint, Θ0c::Ptr{Cdouble}, Cint(P)::Cint, Cint(R)::Cint, tuse_ptr(T_use)::Ptr{Cint},
        Cint(iterations)::Cint, Float64(g_tol)::Cdouble, Cint(max_group_iters)::Cint, Float64(tol)::Cdouble,
        θc::Ptr{Cdouble}, p::Ptr{Cdouble}, init::Ptr{Cdouble}, ll::Ptr{Cdouble}, status::Ptr{Cint},
        nev::Ptr{Clonglong})::Cint)
    (theta_c = θc, p = p, init_c = init, ll = ll, status = status, n_evals = nev[])
end
end # module
