%% antidote_gpu_nif — Erlang side of the MI355X materialization engine.
%%
%% Drop-in for the hot path of clocksi_materializer:materialize/4
%% (src/clocksi_materializer.erl:82-101) and stable_time_functions:get_min_time/1
%% (src/stable_time_functions.erl:51-85).  Terms are encoded here into the SoA
%% binaries of include/antidote_gpu.h; the NIF (antidote_gpu_nif.c) runs the HIP
%% kernels on a dirty scheduler.  Built only where erl_nif.h exists; see
%% INTEGRATION.md for the two-line patches that route the reference through it.
-module(antidote_gpu_nif).

-export([open/1, materialize/6, gst_min/5, select_base/7]).
-export([materialize/4, get_min_time/1]).

-on_load(init/0).

-include("antidote.hrl").

-define(COUNTER, 1).
-define(SET_AW, 2).
-define(REGISTER_MV, 3).
-define(F_NEWSS, 1).
-define(F_CT_IGNORE, 2).
-define(F_ERR_UNEXPECTED, 4).
-define(F_ERR_CORRUPTED, 8).
-define(INVALID_EFFECT, -16#8000000000000000).
-define(U64_MAX, 16#FFFFFFFFFFFFFFFF).

init() ->
    Dir = case code:priv_dir(antidote) of
              {error, _} -> filename:dirname(code:which(?MODULE));
              P -> P
          end,
    erlang:load_nif(filename:join(Dir, "antidote_gpu_nif"), 0).

open(_Device) -> erlang:nif_error(not_loaded).
materialize(_Ctx, _Type, _NDcs, _Log, _Read, _CapOff) -> erlang:nif_error(not_loaded).
gst_min(_Ctx, _NDcs, _NParts, _Clocks, _Defined) -> erlang:nif_error(not_loaded).
select_base(_Ctx, _NDcs, _CacheOff, _Clocks, _ClockMask, _R, _RMask) -> erlang:nif_error(not_loaded).

ctx() ->
    case persistent_term:get({?MODULE, ctx}, undefined) of
        undefined ->
            {ok, C} = open(0),
            persistent_term:put({?MODULE, ctx}, C),
            C;
        C -> C
    end.

type_id(antidote_crdt_counter_pn) -> ?COUNTER;
type_id(antidote_crdt_set_aw) -> ?SET_AW;
type_id(antidote_crdt_register_mv) -> ?REGISTER_MV.

%% ---------------------------------------------------------------------------
%% clocksi_materializer:materialize/4, same arguments and results.
materialize(Type, TxId, MinSnapshotTime,
            #snapshot_get_response{snapshot_time = SCT, ops_list = Ops,
                                   materialized_snapshot = #materialized_snapshot{value = Base}}) ->
    TypeId = type_id(Type),
    OpList = oldest_first(Ops),
    Dcs = dc_table([MinSnapshotTime, SCT | [clock_of(Op) || {_, Op} <- OpList]]),
    D = max(1, length(Dcs)),
    Idx = maps:from_list(lists:zip(Dcs, lists:seq(0, length(Dcs) - 1))),
    {Log, Terms, Tags, Toks} = encode_log(Type, TypeId, OpList, Idx, D),
    {Read, CapOff} = encode_read(TypeId, Idx, D, MinSnapshotTime, SCT, TxId, Base, Log, Tags, Toks),
    {ok, R} = materialize(ctx(), TypeId, D, Log, Read, CapOff),
    decode(Type, TypeId, Dcs, D, R, Terms, Tags, Toks).

oldest_first(Ops) when is_list(Ops) -> lists:reverse(Ops);
oldest_first(Tuple) when is_tuple(Tuple) ->
    {Length, _} = element(2, Tuple),
    [element(?FIRST_OP + I, Tuple) || I <- lists:seq(0, Length - 1)].

clock_of(#clocksi_payload{snapshot_time = SS, commit_time = {Dc, Ct}}) ->
    dict:store(Dc, Ct, SS).

dc_table(Clocks) ->
    lists:usort(lists:append([dict:fetch_keys(C) || C <- Clocks, C =/= ignore])).

row(Clock, Idx, D) ->
    Vals = lists:foldl(fun({Dc, T}, A) -> setelement(maps:get(Dc, Idx) + 1, A, T) end,
                       erlang:make_tuple(D, 0), dict:to_list(Clock)),
    Mask = lists:foldl(fun(Dc, M) -> M bor (1 bsl maps:get(Dc, Idx)) end, 0, dict:fetch_keys(Clock)),
    W = (D + 63) div 64,
    {<< <<V:64/native>> || V <- tuple_to_list(Vals) >>, <<Mask:(64 * W)/little>>}.

encode_log(Type, TypeId, OpList, Idx, D) ->
    N = length(OpList),
    KeyType = case lists:all(fun({_, #clocksi_payload{type = T}}) -> T =:= Type end, OpList) of
                  true -> TypeId;
                  false -> 16#FF
              end,
    {Rows, Masks} = lists:unzip([row(clock_of(Op), Idx, D) || {_, Op} <- OpList]),
    Ids = << <<Id:32/native>> || {Id, _} <- OpList >>,
    TxIds = << <<(erlang:phash2(Op#clocksi_payload.txid, 16#7FFFFFFF) + 1):64/native>> || {_, Op} <- OpList >>,
    Base = {<<0:64/native, N:64/native>>, <<KeyType:8>>, iolist_to_binary(Rows),
            iolist_to_binary(Masks), Ids, TxIds},
    case TypeId of
        ?COUNTER ->
            {Effs, Terms} = lists:foldl(
                fun({_, #clocksi_payload{op_param = E}}, {Acc, T}) when is_integer(E),
                                                                        E > ?INVALID_EFFECT,
                                                                        E < 16#8000000000000000 ->
                        {[<<E:64/signed-native>> | Acc], T};
                   ({_, #clocksi_payload{op_param = E}}, {Acc, T}) ->
                        {[<<?INVALID_EFFECT:64/signed-native>> | Acc], [{length(Acc), E} | T]}
                end, {[], []}, OpList),
            {erlang:append_element(erlang:append_element(
                 erlang:append_element(erlang:append_element(erlang:append_element(Base,
                     iolist_to_binary(lists:reverse(Effs))), <<>>), <<>>), <<>>), <<>>),
             maps:from_list(Terms), #{}, #{}};
        _ ->
            %% one entry per op (add_all / multi-part effects are split by the
            %% Python reference encoder; this shim keeps one part per op)
            encode_tag_log(Base, OpList, TypeId)
    end.

encode_tag_log(Base, OpList, TypeId) ->
    {Tags, Toks, Tag, Add, RemOff, Rem, Terms, _} = lists:foldl(
        fun({_, #clocksi_payload{op_param = E}}, {Tg, Tk, TagA, AddA, OffA, RemA, Tm, I}) ->
                case part(TypeId, E) of
                    {ok, TagTerm, AddTok, Rems} ->
                        {Tg1, TagId} = intern(TagTerm, Tg),
                        {Tk1, AddId} = case AddTok of none -> {Tk, 0}; _ -> intern(AddTok, Tk) end,
                        {Tk2, RemIds} = lists:foldl(fun(X, {T, L}) -> {T2, Id} = intern(X, T), {T2, [Id | L]} end,
                                                    {Tk1, []}, Rems),
                        Off = hd(OffA) + length(RemIds),
                        {Tg1, Tk2, [<<TagId:32/native>> | TagA], [<<AddId:64/native>> | AddA],
                         [Off | OffA], [[<<R:64/native>> || R <- lists:reverse(RemIds)] | RemA], Tm, I + 1};
                    error ->
                        {Tg, Tk, [<<16#FFFFFFFF:32/native>> | TagA], [<<0:64>> | AddA],
                         [hd(OffA) | OffA], RemA, maps:put(I, E, Tm), I + 1}
                end
        end, {#{}, #{}, [], [], [0], [], #{}, 0}, OpList),
    Log = list_to_tuple(tuple_to_list(Base) ++
                        [<<>>, iolist_to_binary(lists:reverse(Tag)), iolist_to_binary(lists:reverse(Add)),
                         << <<O:32/native>> || O <- lists:reverse(RemOff) >>,
                         iolist_to_binary(lists:reverse(Rem))]),
    {Log, Terms, Tags, Toks}.

part(?SET_AW, [{Elem, Adds, Rems}]) when length(Adds) =< 1 ->
    {ok, Elem, case Adds of [A] -> A; [] -> none end, Rems};
part(?REGISTER_MV, {reset, Ovr}) -> {ok, reset, none, Ovr};
part(?REGISTER_MV, {Value, Token, Ovr}) -> {ok, Value, Token, Ovr};
part(_, _) -> error.

intern(Term, Map) ->
    case maps:find(Term, Map) of
        {ok, Id} -> {Map, Id};
        error -> Id = maps:size(Map) + 1, {maps:put(Term, Id, Map), Id}
    end.

encode_read(TypeId, Idx, D, R, SCT, TxId, Base, Log, _Tags, _Toks) ->
    {RRow, RMask} = row(R, Idx, D),
    {SRow, SMask, SIgn} = case SCT of
                              ignore -> {<<>>, <<>>, <<1:8>>};
                              _ -> {Sr, Sm} = row(SCT, Idx, D), {Sr, Sm, <<0:8>>}
                          end,
    Tx = case TxId of ignore -> <<0:64>>; _ -> <<(erlang:phash2(TxId, 16#7FFFFFFF) + 1):64/native>> end,
    BaseValue = case TypeId of ?COUNTER -> <<Base:64/signed-native>>; _ -> <<>> end,
    Read = {<<0:64/native>>, RRow, RMask, SRow, SMask, SIgn, Tx, BaseValue, <<>>, <<>>, <<>>},
    Cap = case TypeId of
              ?COUNTER -> <<>>;
              _ -> N = byte_size(element(8, Log)) div 8, <<0:64/native, N:64/native>>
          end,
    {Read, Cap}.

decode(Type, TypeId, Dcs, D, {Value, Hole, LastCt, LastCtMask, Count, Flags, ErrPos, OutN, OutTag, OutTok},
       Terms, Tags, Toks) ->
    <<F:32/native>> = Flags,
    <<C:32/native>> = Count,
    <<H:64/signed-native>> = Hole,
    if
        F band ?F_ERR_CORRUPTED =/= 0 -> erlang:error(corrupted_ops_cache);
        F band ?F_ERR_UNEXPECTED =/= 0 ->
            <<E:32/native>> = ErrPos,
            {error, {unexpected_operation, maps:get(E, Terms, undefined), Type}};
        true ->
            Ct = case F band ?F_CT_IGNORE of
                     0 -> decode_clock(Dcs, D, LastCt, LastCtMask);
                     _ -> ignore
                 end,
            V = case TypeId of
                    ?COUNTER -> <<X:64/signed-native>> = Value, X;
                    _ -> decode_state(TypeId, OutN, OutTag, OutTok, Tags, Toks)
                end,
            {ok, V, H, Ct, F band ?F_NEWSS =/= 0, C}
    end.

decode_clock(Dcs, D, Vals, MaskBin) ->
    W = (D + 63) div 64,
    <<Mask:(64 * W)/little>> = MaskBin,
    L = [V || <<V:64/native>> <= Vals],
    dict:from_list([{Dc, lists:nth(I + 1, L)} || {Dc, I} <- lists:zip(Dcs, lists:seq(0, length(Dcs) - 1)),
                                                 (Mask bsr I) band 1 =:= 1]).

decode_state(TypeId, <<N:32/native>>, TagBin, TokBin, Tags, Toks) ->
    RTags = maps:from_list([{I, T} || {T, I} <- maps:to_list(Tags)]),
    RToks = maps:from_list([{I, T} || {T, I} <- maps:to_list(Toks)]),
    Pairs = lists:sublist(lists:zip([T || <<T:32/native>> <= TagBin], [K || <<K:64/native>> <= TokBin]), N),
    Terms = [{maps:get(T, RTags), maps:get(K, RToks)} || {T, K} <- Pairs],
    case TypeId of
        ?SET_AW ->
            orddict:from_list(lists:foldr(fun({E, K}, Acc) ->
                                                  orddict:update(E, fun(L) -> [K | L] end, [K], Acc)
                                          end, [], Terms));
        ?REGISTER_MV -> lists:sort(Terms)
    end.

%% ---------------------------------------------------------------------------
%% stable_time_functions:get_min_time/1 on the device.
get_min_time(Dict) ->
    Entries = dict:to_list(Dict),
    Dcs = lists:usort(lists:append([dict:fetch_keys(V) || {_, V} <- Entries, V =/= undefined])),
    D = max(1, length(Dcs)),
    Rows = [case V of
                undefined -> << <<?U64_MAX:64/native>> || _ <- lists:seq(1, D) >>;
                _ -> << <<(case dict:find(Dc, V) of {ok, T} -> T; error -> ?U64_MAX end):64/native>>
                        || Dc <- Dcs >>
            end || {_, V} <- Entries],
    Defined = << <<(case V of undefined -> 0; _ -> 1 end):8>> || {_, V} <- Entries >>,
    {ok, Vec} = gst_min(ctx(), D, length(Entries), iolist_to_binary(Rows), Defined),
    Words = [W || <<W:64/native>> <= Vec],
    dict:from_list([{Dc, T} || {Dc, T} <- lists:zip(Dcs, lists:sublist(Words, length(Dcs))),
                               T =/= ?U64_MAX]).
