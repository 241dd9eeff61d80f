# Julia @ccall binding of libyfm_hip.so (include/yfm.h). Not executable in this image (no julia).
# See INTEGRATION.md for the drop-in get_loss / compute_loss_batch methods.
module YFMAMD
const LIB = get(ENV, "YFM_LIB", joinpath(@__DIR__, "..", "yfm_amd", "libyfm_hip.so"))

const YFM_MODEL_DNS, YFM_MODEL_TVL, YFM_MODEL_GNS5 = Cint(0), Cint(1), Cint(2)
const UNCONSTRAINED, CONSTRAINED = Cint(0), Cint(1)

struct YFMError <: Exception; code::Cint; msg::String; end
check(rc) = rc == 0 || throw(YFMError(rc, unsafe_string(@ccall LIB.yfm_last_error()::Cstring)))

mutable struct Context
    ptr::Ptr{Cvoid}
    panel_id::UInt     # objectid of the last uploaded panel
    function Context(device::Integer = 0)
        p = @ccall LIB.yfm_create(Cint(device)::Cint)::Ptr{Cvoid}
        p == C_NULL && throw(YFMError(-2, unsafe_string(@ccall LIB.yfm_last_error()::Cstring)))
        ctx = new(p, 0)
        finalizer(c -> @ccall(LIB.yfm_destroy(c.ptr::Ptr{Cvoid})::Cvoid), ctx)
    end
end
const CTX = Ref{Context}()
ctx() = isassigned(CTX) ? CTX[] : (CTX[] = Context(0))

function set_panel!(c::Context, data::Matrix{Float64}, maturities::Vector{Float64})
    N, T = size(data)                       # N×T column-major, as load_data returns it
    GC.@preserve data maturities check(@ccall LIB.yfm_set_panel(c.ptr::Ptr{Cvoid}, data::Ptr{Cdouble},
        Cint(N)::Cint, Cint(T)::Cint, maturities::Ptr{Cdouble})::Cint)
    c.panel_id = objectid(data)
end

kind(::YieldFactorModels.AbstractDNSModel) = YFM_MODEL_DNS
kind(::YieldFactorModels.AbstractTVλDNSModel) = YFM_MODEL_TVL

"Batched loglik: Θ is P×B (one candidate per column).  space: UNCONSTRAINED (compute_loss input) or CONSTRAINED (set_params! input)."
function loglik_batch(model, data::Matrix{Float64}, Θ::Matrix{Float64}; space = UNCONSTRAINED,
                      T_use::Union{Nothing,Vector{Cint}} = nothing)
    c = ctx()
    c.panel_id == objectid(data) || set_panel!(c, data, Vector{Float64}(model.base.maturities))
    P, B = size(Θ)
    out = Vector{Float64}(undef, B)
    tu = T_use === nothing ? C_NULL : pointer(T_use)
    GC.@preserve Θ out T_use check(@ccall LIB.yfm_loglik_batch(c.ptr::Ptr{Cvoid}, kind(model)::Cint, space::Cint,
        Θ::Ptr{Cdouble}, Cint(P)::Cint, Cint(B)::Cint, tu::Ptr{Cint}, out::Ptr{Cdouble})::Cint)
    out                                        # +loglik per column; -Inf / NaN as documented in yfm.h
end
end # module
