% demo_registration.m - the MEX call sequence of the reference's demo
% (test_opticalflow2d.m:42-59) against the MI355X build: build the gateway
% first with opticalflow2d_amd/mex/compile_mex_function.m (needs Octave or
% MATLAB, which this repository's CI image does not have; the same sequence runs
% from Python in examples/demo_registration.py).
%
% Synthetic inputs: a bright disk and the same disk shifted by (4, 2) pixels.

n = 256;
[x, y] = ndgrid(0:n-1, 0:n-1);
r = n / 4;
Iref = double((x - n/2).^2 + (y - n/2).^2 <= r^2);
Imov = double((x - n/2 - 4).^2 + (y - n/2 - 2).^2 <= r^2);

pad = 11;                                   % replicate-pad x by 11 pixels
Iref = [repmat(Iref(1, :), pad, 1); Iref; repmat(Iref(end, :), pad, 1)];
Imov = [repmat(Imov(1, :), pad, 1); Imov; repmat(Imov(end, :), pad, 1)];
[dimx, dimy] = size(Iref);

niter = [25 25 200];                        % one entry per scale (nscales + 1)
nscales = 2;
nrefine = 1;
params = [0.25 0.0];                        % fluid: mu, lambda
regularisation = 5;                         % SolverOptions.h: 0 diffusion, 1 curvature,
                                            % 2 elastic, 3 Thirion, 4 diffeomorphic, 5 fluid
verbose = 0;

OpticalFlow2d([dimx, dimy], niter, nscales, regularisation, ...
              params, numel(params), nrefine, verbose);   % init
t0 = tic();
OpticalFlow2d(Iref, Imov);                                % register
elapsed = toc(t0);
motion = OpticalFlow2d();                                 % [dimx dimy 2]
Ireg = OpticalFlow2d(Imov);                               % warped moving image
OpticalFlow2d();                                          % close

core_x = 1+pad:dimx-pad;
core_y = 1+pad:dimy-pad;
m = motion(core_x, core_y, :);
printf("registration: %.3f s\n", elapsed);
printf("Distribution: %.3f +/ %.3f\n", mean(m(:)), std(m(:)));
printf("Maxabs: %.3f\n", max(abs(m(:))));
printf("mean |Iref - Imov| %.4f -> mean |Iref - Ireg| %.4f\n", ...
       mean(mean(abs(Iref(core_x, core_y) - Imov(core_x, core_y)))), ...
       mean(mean(abs(Iref(core_x, core_y) - Ireg(core_x, core_y)))));
